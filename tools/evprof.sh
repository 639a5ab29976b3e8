cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/evprof -o ev -- python tools/eval_one.py market1501 20 > gpurun_out/evprof.log 2>&1
