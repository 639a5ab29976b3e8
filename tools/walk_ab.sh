cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
W="--warm 60 --walk 1,4,2,1,4,2,8"
timeout -k 10 120 python tools/gemm_one.py 216064 3072 768 1 20 fold $W > gpurun_out/walk2.log 2>&1 &&
timeout -k 10 120 python tools/gemm_one.py 216064 2304 768 0 20 fold $W >> gpurun_out/walk2.log 2>&1 &&
timeout -k 10 120 python tools/gemm_one.py 216064 768 3072 6 20 $W >> gpurun_out/walk2.log 2>&1 &&
timeout -k 10 120 python tools/gemm_one.py 216064 768 768 6 20 $W >> gpurun_out/walk2.log 2>&1 &&
for w in 1 4; do for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_w${w}_$c -o p -- python tools/gemm_one.py 216064 3072 768 1 5 fold --walk $w > gpurun_out/pmc_w${w}_$c.log 2>&1 || exit 1; done; done
