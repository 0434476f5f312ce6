set -o pipefail
mkdir -p gpurun_out/ab
A="--cpu-seconds 0 --pcie-steps 0 --no-warm-batch --steps 20"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 && \
for r in 1 2; do
for v in split skew1; do
  if [ $v = split ]; then L=sesam-duke-microservice_amd/build/libdukehip.so; else L=sesam-duke-microservice_amd/build/var/libdukehip_$v.so; fi
  DUKEHIP_LIB=$L timeout -k 10 300 python -u bench.py $A > gpurun_out/ab/dd_${v}_$r.log 2>&1 || exit 1
done
done
for v in split skew1; do
  if [ $v = split ]; then L=sesam-duke-microservice_amd/build/libdukehip.so; else L=sesam-duke-microservice_amd/build/var/libdukehip_$v.so; fi
  DUKEHIP_LIB=$L timeout -k 10 300 python -u bench.py --cpu-seconds 0 --pcie-steps 0 --no-warm-batch --workload allpairs --steps 3 > gpurun_out/ab/ap_$v.log 2>&1 || exit 1
done
