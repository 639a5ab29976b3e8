set -o pipefail
mkdir -p gpurun_out/r06s
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_encoder.py -m gpu -k "gemm" > gpurun_out/r06s/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06s/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/walk_ab.py 3 > gpurun_out/r06s/walk_ab.txt 2>&1
rc=$?; echo "walk rc=$rc"; grep -v amdgpu.ids gpurun_out/r06s/walk_ab.txt
exit $rc
