set -e
export TMPDIR=/tmp
V=sesam-duke-microservice_amd/build/var
for wl in dedup longtext; do
for lib in sesam-duke-microservice_amd/build/libdukehip.so $V/libdukehip_bias0.so $V/libdukehip_bias100.so sesam-duke-microservice_amd/build/libdukehip.so; do
  DUKEHIP_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --workload $wl --steps 5 --cpu-seconds 0 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$wl', '$lib'.split('/')[-1], round(d['ms_per_step'],2), round(d['roofline']['avg_launch_ms'],3), flush=True)"
done; done
