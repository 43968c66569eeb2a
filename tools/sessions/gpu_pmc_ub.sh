#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
cat > /tmp/ctr.txt <<'EOT'
pmc: FETCH_SIZE
pmc: TCC_HIT_sum TCC_MISS_sum
pmc: TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
pmc: SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD
pmc: TA_TA_BUSY_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
pmc: TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
pmc: GRBM_GUI_ACTIVE
EOT
timeout -k 10 300 rocprofv3 -i /tmp/ctr.txt --kernel-trace -d gpurun_out/pmc_ub2 -o pmc --output-format csv -- python tools/ubench.py part > gpurun_out/pmc_ub2.log 2>&1; echo rc=$?
