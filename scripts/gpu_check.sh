set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== smoke" 
timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"
tail -3 gpurun_out/smoke.log
echo "== gpu tests"
timeout -k 10 900 python -m pytest tests/test_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_gpu.log
