set -o pipefail
mkdir -p gpurun_out/pp
export TMPDIR=/tmp
for P in DOB ADDRESS NAME DOB,ADDRESS,NAME; do
  PROPS=$P timeout -s KILL 240 rocprofv3 --kernel-include-regex "k_score" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/pp/$P -o pmc -- python3 scripts/ablate_props.py > gpurun_out/pp/$P.log 2>&1 || exit 1
done
