# The reference sweep config's learning curve on the device, both stand-in layouts (scripts/learning_curve.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lc
for L in cities grid; do
  timeout -k 10 600 python -u scripts/learning_curve.py gpurun_out/lc/lc_$L.json --layout $L --chunk 1000 > gpurun_out/lc/lc_$L.log 2>&1; rc=$?
  echo "layout $L rc=$rc"; tail -1 gpurun_out/lc/lc_$L.log
  [ $rc -eq 0 ] || exit $rc
done
