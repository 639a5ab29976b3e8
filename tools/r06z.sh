set -o pipefail
mkdir -p gpurun_out/r06z
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r06z/pytest_gpu.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06z/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r06z/smoke.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06z/bench.json 2> gpurun_out/r06z/bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.loads(open('gpurun_out/r06z/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['files_to_map']['wall_s'], d['backend']['eval_rows']['frac'], d['backend']['distmat_f16']['ms'])"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06z/prof -o bench -- python3 bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/r06z/bench_under_rocprof.json 2> gpurun_out/r06z/prof.err
rc=$?; echo "prof rc=$rc"
find gpurun_out/r06z/prof -name "*kernel_trace.csv" -delete
exit $rc
