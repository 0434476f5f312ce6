set -o pipefail
mkdir -p gpurun_out
nproc > gpurun_out/ingest.log; cat /sys/fs/cgroup/cpu.max >> gpurun_out/ingest.log 2>&1
timeout -k 10 300 python -u scripts/bench_ingest.py >> gpurun_out/ingest.log 2>&1
