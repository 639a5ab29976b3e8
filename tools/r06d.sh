set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_encoder.py -m gpu -k "mhsa" > gpurun_out/r06d/pytest_mhsa.txt 2>&1
rc=$?; echo "pytest_mhsa rc=$rc"; tail -4 gpurun_out/r06d/pytest_mhsa.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_rr_ab.py 3 > gpurun_out/r06d/attn_rr_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06d/attn_rr_ab.txt | tail -12
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_encoder.py tests/test_gpu_pipeline.py -m gpu > gpurun_out/r06d/pytest_enc.txt 2>&1
rc=$?; echo "enc rc=$rc"; tail -3 gpurun_out/r06d/pytest_enc.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-msmt17 --no-rerank --no-text --no-cpu-baseline --no-backend --no-preprocess --no-jpeg --no-files > gpurun_out/r06d/bench.json 2> gpurun_out/r06d/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/r06d/bench.json
