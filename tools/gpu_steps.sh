#!/bin/bash
# Runs named GPU steps in order on the box, each under its own time limit,
# stopping at the first failure (no retries).  Logs: gpurun_out/<tag>/<step>.log
# Usage: tools/gpu_steps.sh TAG step[,step...]
#   steps: pytest smoke bench bench_c4 bench_c5 stats_c2 stats_c3 stats_c4 stats_c5
#          stats_route stats_compact pmc_c2 pmc_c3 pmc_c4 pmc_c5 (and the experiments below)
set -o pipefail
TAG=${1:?tag}; STEPS=${2:?steps}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-400
  return $rc
}
pmc() {  # workload counter benchargs...
  local w=$1 c=$2; shift 2
  run "pmc_${w}_$c" 150 timeout -s KILL 140 rocprofv3 --pmc "$c" --kernel-trace \
      -d "$OUT/pmc_${w}_$c" -o pmc --output-format csv -- python bench.py "$@"
}
python -c "import sys; sys.path.insert(0, '.'); import bench; print('library kernel sha', bench.library_kernel_sha(), 'sources', bench.kernel_source_sha())" 2>/dev/null | tee "$OUT/library.txt"
for s in ${STEPS//,/ }; do
  case $s in
    pytest) run pytest 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) run bench 600 python bench.py || exit 1 ;;
    bench_quick) run bench_quick 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline || exit 1 ;;
    bench_c4) run bench_c4 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1 ;;
    bench_c4w) run bench_c4w 400 python bench.py --workload c4w --steps 5 --warmup 1 --no-extras --no-cpu-baseline || exit 1 ;;
    ub_prim) run ub_prim 200 python tools/ubench.py || exit 1 ;;
    ub_isa) run ub_isa 120 python tools/ubench_isa.py || exit 1 ;;
    ub_part) run ub_part 300 python tools/ubench.py part || exit 1 ;;
    ub_part_c5) run ub_part_c5 300 python tools/ubench.py part_c5 || exit 1 ;;
    ub_part_c4) run ub_part_c4 300 python tools/ubench.py part_c4 || exit 1 ;;
    ub_p2ab) run ub_p2ab 300 python tools/ubench.py p2ab || exit 1 ;;
    ub_p2ab_c5) run ub_p2ab_c5 300 python tools/ubench.py p2ab_c5 || exit 1 ;;
    ub_p2ab_c4) run ub_p2ab_c4 300 python tools/ubench.py p2ab_c4 || exit 1 ;;
    sq_part_c4) run sq_part_c4_a 200 timeout -s KILL 190 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$OUT/sq_part_c4_a" -o pmc --output-format csv -- python tools/ubench.py part_c4 || exit 1
             run sq_part_c4_b 200 timeout -s KILL 190 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/sq_part_c4_b" -o pmc --output-format csv -- python tools/ubench.py part_c4 || exit 1 ;;
    ub_stack) run ub_stack 300 python tools/ubench.py stack || exit 1 ;;
    build_ab_c2) run build_ab_c2 400 python tools/build_ab.py 5 c2 || exit 1 ;;
    build_ab_c5) run build_ab_c5 400 python tools/build_ab.py 3 c5 || exit 1 ;;
    build_ab_f10) run build_ab_f10 400 python tools/build_ab.py 3 f10 || exit 1 ;;
    ub_p1abl) run ub_p1abl 300 python tools/ubench.py p1abl || exit 1 ;;
    ub_p1tail) run ub_p1tail 300 python tools/ubench.py p1tail || exit 1 ;;
    sq_p1abl) run sq_p1abl_a 200 timeout -s KILL 190 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$OUT/sq_p1abl_a" -o pmc --output-format csv -- python tools/ubench.py p1abl || exit 1
              run sq_p1abl_b 200 timeout -s KILL 190 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/sq_p1abl_b" -o pmc --output-format csv -- python tools/ubench.py p1abl || exit 1 ;;
    pcie) run pcie 120 python tools/pcie_probe.py || exit 1 ;;
    ub_ladder) run ub_ladder 300 python tools/ubench.py ladder || exit 1 ;;
    ub_chunks) run ub_chunks 300 env UB_LADDER=2,201,202,203,204,206,208 python tools/ubench.py ladder || exit 1 ;;
    ub_p1ab) run ub_p1ab 300 python tools/ubench.py p1ab || exit 1 ;;
    sq_part) run sq_part_a 150 timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$OUT/sq_part_a" -o pmc --output-format csv -- python tools/ubench.py part || exit 1
             run sq_part_b 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/sq_part_b" -o pmc --output-format csv -- python tools/ubench.py part || exit 1
             run sq_part_c 150 timeout -s KILL 140 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$OUT/sq_part_c" -o pmc --output-format csv -- python tools/ubench.py part || exit 1 ;;
    sq_c3) run sq_c3_a 150 timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$OUT/sq_c3_a" -o pmc --output-format csv -- python tools/probe_prof.py auto 10 || exit 1
           run sq_c3_b 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/sq_c3_b" -o pmc --output-format csv -- python tools/probe_prof.py auto 10 || exit 1 ;;
    bench_c5) run bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-extras --no-cpu-baseline || exit 1 ;;
    stats_c2) run stats_c2 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_c2" -o run --output-format csv -- python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1 ;;
    stats_c4) run stats_c4 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_c4" -o run --output-format csv -- python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1 ;;
    stats_c5) run stats_c5 400 rocprofv3 --kernel-trace --stats -d "$OUT/stats_c5" -o run --output-format csv -- python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1 ;;
    probe_sweep) run probe_sweep 300 python tools/probe_sweep.py || exit 1 ;;
    probe_ab) run probe_ab 400 python tools/probe_ab.py 3 || exit 1 ;;
    ab_c2) run ab_c2 600 bash tools/ab.sh "$TAG/ab_c2" 3 --no-extras --steps 200 --warmup 20 || exit 1 ;;
    ab_full) run ab_full 900 bash tools/ab.sh "$TAG/ab_full" 2 --no-c4 --no-c5 --steps 100 --warmup 10 || exit 1 ;;
    ab_c5) run ab_c5 600 bash tools/ab.sh "$TAG/ab_c5" 2 --workload c5 --no-extras --steps 20 --warmup 3 || exit 1 ;;
    stats_compact) run stats_compact 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_compact" -o run --output-format csv -- python tools/compact_prof.py 40 || exit 1 ;;
    stats_compact_alt) run stats_compact_alt 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_compact_alt" -o run --output-format csv -- python tools/compact_prof.py 40 alt || exit 1 ;;
    stats_c3_alt) run stats_c3_alt 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_c3_alt" -o run --output-format csv -- python tools/probe_prof.py auto 30 alt || exit 1 ;;
    stats_route) run stats_route 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_route" -o run --output-format csv -- python tools/probe_prof.py route 30 || exit 1 ;;
    stats_f10) run stats_f10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_f10" -o run --output-format csv -- python tools/probe_prof.py auto 30 - f10 || exit 1 ;;
    stats_route_f10) run stats_route_f10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_route_f10" -o run --output-format csv -- python tools/probe_prof.py route 30 - f10 || exit 1 ;;
    bench_rep) run bench_rep1 600 python bench.py || exit 1
               run bench_rep2 600 python bench.py || exit 1 ;;
    sq_route) for w in c3 f10; do
                run sq_route_${w}_a 150 timeout -s KILL 140 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$OUT/sq_route_${w}_a" -o pmc --output-format csv -- python tools/probe_prof.py route 10 - $w || exit 1
                run sq_route_${w}_b 150 timeout -s KILL 140 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d "$OUT/sq_route_${w}_b" -o pmc --output-format csv -- python tools/probe_prof.py route 10 - $w || exit 1
              done ;;
    stats_c3) run stats_c3 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_c3" -o run --output-format csv -- python tools/probe_prof.py auto 30 || exit 1 ;;
    pmc_c2) pmc c2 FETCH_SIZE --steps 10 --warmup 2 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1
            pmc c2 WRITE_SIZE --steps 10 --warmup 2 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1 ;;
    pmc_c4) pmc c4 FETCH_SIZE --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1
            pmc c4 WRITE_SIZE --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1 ;;
    pmc_c3) run pmc_c3_FETCH_SIZE 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/pmc_c3_FETCH_SIZE" -o pmc --output-format csv -- python tools/probe_prof.py auto 10 || exit 1
            run pmc_c3_WRITE_SIZE 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/pmc_c3_WRITE_SIZE" -o pmc --output-format csv -- python tools/probe_prof.py auto 10 || exit 1 ;;
    bench_dist2) run bench_dist2 600 env BLOOMHIP_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline || exit 1 ;;
    bench_driver) run bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1 ;;
    cal) run cal 120 python tools/ubench.py cal || exit 1
         for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum" \
                  "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
           n=$(echo $c | cut -d' ' -f1)
           run "cal_$n" 150 timeout -s KILL 140 rocprofv3 --pmc $c --kernel-trace -d "$OUT/cal_$n" -o pmc --output-format csv -- python tools/ubench.py cal || exit 1
         done ;;
    pmc_c5) pmc c5 FETCH_SIZE --workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1
            pmc c5 WRITE_SIZE --workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-extras --prewarm-s 0 || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "all steps ok"
