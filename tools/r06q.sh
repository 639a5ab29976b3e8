set -o pipefail
mkdir -p gpurun_out/r06q
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_rerank.py tests/test_gpu_rerank_sharded.py tests/test_gpu_scale.py tests/test_gpu_pipeline.py -m gpu > gpurun_out/r06q/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06q/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06q/prof -o distf16 -- python3 tools/distf16_prof.py > gpurun_out/r06q/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-files > gpurun_out/r06q/bench.json 2> gpurun_out/r06q/bench.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/r06q/bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['backend']))"
exit $rc
