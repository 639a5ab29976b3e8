set -o pipefail
mkdir -p gpurun_out/r06i
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r06i/pytest_gpu.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06i/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06i/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r06i/smoke.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06i/bench.json 2> gpurun_out/r06i/bench.err
rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.loads(open('gpurun_out/r06i/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['files_to_map']['wall_s'], d['msmt17']['end_to_end_wall_s'])"
timeout -k 10 700 python -u tools/rerank_scale_oracle.py msmt17 16 > gpurun_out/r06i/rerank_msmt17_vs_oracle.txt 2>&1
rc=$?; echo "msmt17 oracle rc=$rc"; tail -2 gpurun_out/r06i/rerank_msmt17_vs_oracle.txt
