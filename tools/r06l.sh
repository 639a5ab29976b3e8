set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_backend.py tests/test_gpu_scale.py tests/test_gpu_sharded_surface.py -m gpu > gpurun_out/r06l/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06l/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/eval_ab.py tools/ablibs/libreidmi_evold.so,tools/ablibs/libreidmi_evnew.so,tools/ablibs/libreidmi_evcsr.so 3 > gpurun_out/r06l/eval_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06l/eval_ab.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for a in "market1501" "market1501 clustered" "msmt17"; do
  timeout -k 10 120 python -u tools/eval_stamps.py tools/ablibs/libreidmi_evcsrst.so $a > gpurun_out/r06l/stamps.txt 2>&1
  rc=$?; echo "== $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r06l/stamps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
