set -o pipefail
mkdir -p gpurun_out
DK_HOST_TIMING=1 DK_INGEST_TIMING=1 timeout -k 10 400 python -u bench.py --cpu-seconds 0 --pcie-steps 0 > gpurun_out/bench.log 2>&1
