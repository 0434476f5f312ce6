set -o pipefail
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o tr -- python3 bench.py --cpu-seconds 0 --pcie-steps 0 --no-warm-batch --no-json-batch > gpurun_out/trace/bench.log 2>&1
