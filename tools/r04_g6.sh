# C5 ring-depth variants (wrap fixed) and per-kernel training profiles of the two-kernel path
# vs the fused kernels.
mkdir -p gpurun_out
R=$(pwd)
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r04_$name.log" 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  case $rc in 124|134|137|139) echo "stopping after $name"; tail -20 "gpurun_out/r04_$name.log"; exit $rc;; esac
  return 0
}
step c5_variants2 300 python -u tests/diag/c5_variants.py q16 q24 q24k q22 q16
export TMPDIR=/tmp
PNTF_TT_FUSED=2 PNTF_TT_BWD=0 step prof_train_2kernel 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train_2k -o train --output-format csv -- python3 $R/tools/train_profile.py 10000
PNTF_TT_FUSED=3 PNTF_TT_BWD=1 step prof_train_fused 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train_fu -o train --output-format csv -- python3 $R/tools/train_profile.py 10000
