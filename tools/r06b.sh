set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_rerank_oracle_scale.py tests/test_gpu_loader.py tests/test_jpeg.py -m gpu -s > gpurun_out/r06b/pytest_new.txt 2>&1
rc=$?; echo "pytest_new rc=$rc"; tail -3 gpurun_out/r06b/pytest_new.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-msmt17 --no-rerank --no-text --no-cpu-baseline --no-backend --no-preprocess > gpurun_out/r06b/bench_files.json 2> gpurun_out/r06b/bench_files.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r06b/bench_files.json
