set -o pipefail
mkdir -p gpurun_out/r06j
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_loader_sharded.py tests/test_gpu_pipeline.py -m gpu > gpurun_out/r06j/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06j/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/eval_ab.py tools/ablibs/libreidmi_evold.so,tools/ablibs/libreidmi_evnew.so 3 > gpurun_out/r06j/eval_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; cat gpurun_out/r06j/eval_ab.txt | grep -v amdgpu.ids
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-files > gpurun_out/r06j/bench.json 2> gpurun_out/r06j/bench.err
rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/r06j/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['backend']['eval_rows'])"
exit $rc
