# Round-end evidence on one GPU: the -m gpu suite, the wide-kernel profiles (stats + PMC, so
# profiles/pmc_tau_grad.json carries the stamp of this build), then the default bench line.
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/profile_round.sh
echo PROFILED
