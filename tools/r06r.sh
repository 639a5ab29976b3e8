set -o pipefail
mkdir -p gpurun_out/r06r
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06r/prof -o step -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rerank --no-msmt17 --no-text --no-jpeg --no-backend --no-preprocess --no-files > gpurun_out/r06r/bench.json 2> gpurun_out/r06r/bench.err
rc=$?; echo "prof rc=$rc"; tail -c 300 gpurun_out/r06r/bench.json
f=$(find gpurun_out/r06r/prof -name "*kernel_trace.csv" | head -1); echo $f
python3 tools/trace_gaps.py $f > gpurun_out/r06r/gaps.txt; cat gpurun_out/r06r/gaps.txt | head -40
rm -f $f
exit $rc
