set -o pipefail
mkdir -p gpurun_out/r06v
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_encoder.py -m gpu > gpurun_out/r06v/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06v/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/qkv_lib_ab.py tools/ablibs/libreidmi_qkvold.so,tools/ablibs/libreidmi_qkvnew.so 19281 3 > gpurun_out/r06v/qkv_ab.txt 2>&1
rc=$?; echo "qkv rc=$rc"; grep -v amdgpu.ids gpurun_out/r06v/qkv_ab.txt
exit $rc
