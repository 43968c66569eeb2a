#!/bin/bash
# First GPU session: smoke, parity tests, primitive prices, a short bench.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; date +%T
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; tail -5 "gpurun_out/$name.log"
  return $rc
}
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
step pytest_gpu 900 python -m pytest tests -q -m gpu --timeout 300 -p no:cacheprovider
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step ubench 300 python tools/ubench.py || exit 1
step bench 400 python bench.py --steps 20 --warmup 3 || exit 1
