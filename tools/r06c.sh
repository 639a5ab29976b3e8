set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_loader.py -m gpu -s > gpurun_out/r06c/pytest_loader.txt 2>&1
rc=$?; echo "pytest_loader rc=$rc"; tail -3 gpurun_out/r06c/pytest_loader.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/eval_ab.py tools/ablibs/libreidmi_ev_base.so,tools/ablibs/libreidmi_ev_noatomic.so 3 > gpurun_out/r06c/eval_atomic_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; tail -6 gpurun_out/r06c/eval_atomic_ab.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/r06c/pytest_gpu.txt 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 gpurun_out/r06c/pytest_gpu.txt
