# Epilogue cost A/B on the encoder's GEMM shapes (random operands): plain vs non-temporal
# epilogue stores, the same M x N x K with different epilogues, and K = 3072 (epilogue / 4).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/epi_cost.log
W="--warm 40"
: > $O
for spec in "3072 768 1 fold" "3072 768 0" "3072 768 5" "3072 3072 1 fold" \
            "768 768 6" "768 3072 6" "2304 768 0 fold"; do
  set -- $spec
  timeout -k 10 120 python tools/gemm_one.py 216064 $1 $2 $3 20 $4 $W >> $O 2>&1 || exit 1
done
