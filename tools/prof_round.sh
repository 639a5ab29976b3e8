#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of the default bench command, then PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md "rocprofv3 PMC slots") on the
# bench's dominant kernel (ln_2-folded fp16 c_fc GEMM + QuickGELU at the bench batch,
# M = BATCH * 211 token rows; default 19281 = the bench's one encoder call per pass at Market size),
# SQ instruction counts of c_fc and out_proj (tools/isa_budget.py --pmc turns them into a
# per-wave per-tile budget), and SQ counter passes on the vision attention.  Output under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
M=$(( ${BATCH:-19281} * 211 ))
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- \
  python bench.py ${BENCH_ARGS} > gpurun_out/bench_under_rocprof.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$c -o p -- \
    python tools/gemm_one.py $M 3072 768 1 5 fold > gpurun_out/pmc_$c.log 2>&1
done
# c_fc SQ / GRBM passes: MFMA busy and the clock the chip holds under this load
# (GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall, MI355X_MICROARCH.md "DVFS give-back")
j=0
for cs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
          "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  j=$((j + 1))
  timeout -s KILL 90 rocprofv3 --pmc $cs --kernel-trace --output-format csv -d gpurun_out/cfc_pmc$j -o p -- \
    python tools/gemm_one.py $M 3072 768 1 20 fold > gpurun_out/cfc_pmc$j.log 2>&1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d gpurun_out/outp_pmc -o p -- \
  python tools/gemm_one.py $M 768 768 6 20 > gpurun_out/outp_pmc.log 2>&1
i=0
for cs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
          "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $cs --kernel-trace --output-format csv -d gpurun_out/attn_pmc$i -o p -- \
    python tools/attn_one.py 5 > gpurun_out/attn_pmc$i.log 2>&1
done
