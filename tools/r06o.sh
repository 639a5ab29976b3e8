set -o pipefail
mkdir -p gpurun_out/r06o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_encoder.py tests/test_gpu_rerank.py -m gpu > gpurun_out/r06o/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06o/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-files > gpurun_out/r06o/bench.json 2> gpurun_out/r06o/bench.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/r06o/bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['backend']))"
exit $rc
