set -o pipefail
mkdir -p gpurun_out/r06x
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_loader.py tests/test_gpu_loader_sharded.py tests/test_gpu_scale.py -m gpu > gpurun_out/r06x/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06x/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/eval_ab.py tools/ablibs/libreidmi_evprep0.so,tools/ablibs/libreidmi_evprep1.so 3 > gpurun_out/r06x/eval_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06x/eval_ab.txt | grep "^r2"
exit $rc
