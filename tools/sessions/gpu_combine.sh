#!/bin/bash
# combine workgroup size and C3 run-table layout A/B, plus parity
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-4} | cut -c1-400
  return $rc
}
step pytest_gpu 600 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread || exit 1
prof() { # tag, env...
  local tag=$1; shift
  env "$@" TMPDIR=/tmp timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cb_$tag -o run --output-format csv -- python tools/probe_prof.py auto 30 > gpurun_out/cb_$tag.log 2>&1
}
for cfg in "c512 BLOOMHIP_COMBINE_BLOCK=512" "c1024 BLOOMHIP_COMBINE_BLOCK=1024" "c256 BLOOMHIP_COMBINE_BLOCK=256" "rows BLOOMHIP_COLUMN_TABLE_MAX=8000000"; do
  set -- $cfg
  echo "== prof $1"; prof "$@" || exit 1
done
echo done
