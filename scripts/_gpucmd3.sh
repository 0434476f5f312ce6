set -o pipefail
mkdir -p gpurun_out/ab
V=sesam-duke-microservice_amd/build/var/libdukehip_skew1.so
A="--cpu-seconds 0 --pcie-steps 0 --no-warm-batch"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A > gpurun_out/ab/dd_pk2.log 2>&1 && \
DUKEHIP_LIB=$V timeout -k 10 300 python -u bench.py $A > gpurun_out/ab/dd_skew1.log 2>&1 && \
timeout -k 10 300 python -u bench.py $A --workload allpairs --steps 3 > gpurun_out/ab/ap_pk2.log 2>&1 && \
DUKEHIP_LIB=$V timeout -k 10 300 python -u bench.py $A --workload allpairs --steps 3 > gpurun_out/ab/ap_skew1.log 2>&1
