#!/bin/bash
# Round-end check on the GPU box: the full GPU test suite, smoke(), and the bench line (the
# driver's command). Stops at the first failing step. Outputs under gpurun_out/final/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/final
step() {
  local label=$1 tmo=$2; shift 2
  echo "=== [$label] $(date +%T)"
  timeout -k 10 "$tmo" "$@" > gpurun_out/final/$label.out 2> gpurun_out/final/$label.err
  local rc=$?
  echo "=== [$label] rc=$rc"; tail -n 3 gpurun_out/final/$label.out
  [ $rc -eq 0 ] || exit $rc
}
step gputests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py --steps 20 --warmup 5
