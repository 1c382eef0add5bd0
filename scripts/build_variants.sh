# Tuning builds of libsfl.so from the current sources (same build id): SFL_PROFILE phase cycles,
# SFL_AB_* store-drop timing builds.  Usage: bash scripts/build_variants.sh PROFILE AB_NO_QST ...
cd "$(dirname "$0")/../network-distributed-q-learning_amd"
for v in "$@"; do
  python -c "import build; build.build_hip(out='libsfl_$(echo $v | tr A-Z a-z).so', defines=['SFL_$v'], force=True)" 2>/dev/null &
done
wait
ls -la libsfl_*.so
