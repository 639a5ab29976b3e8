#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of the default bench command, then PMC passes
# (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md "rocprofv3 PMC slots") on the
# bench's dominant kernel (ln_2-folded fp16 c_fc GEMM + QuickGELU, M = 1024*211, the bench batch).  Output under gpurun_out/.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- \
  python bench.py ${BENCH_ARGS} > gpurun_out/bench_under_rocprof.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$c -o p -- \
    python tools/gemm_one.py 216064 3072 768 1 5 fold > gpurun_out/pmc_$c.log 2>&1
done
