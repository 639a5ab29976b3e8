set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_encoder.py -m gpu -k "mhsa" > gpurun_out/r06g/pytest_mhsa.txt 2>&1
rc=$?; echo "pytest_mhsa rc=$rc"; tail -3 gpurun_out/r06g/pytest_mhsa.txt
if [ $rc -ne 0 ]; then exit $rc; fi
BENCH_ARGS="" timeout -k 10 1000 bash tools/prof_round.sh > gpurun_out/r06g/prof_round.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -5 gpurun_out/r06g/prof_round.log; tail -c 400 gpurun_out/bench_under_rocprof.json
