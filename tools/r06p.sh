set -o pipefail
mkdir -p gpurun_out/r06p
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_backend.py -m gpu -k "distmat" > gpurun_out/r06p/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06p/pytest.txt
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06p/prof -o distf16 -- python3 tools/distf16_prof.py > gpurun_out/r06p/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; find gpurun_out/r06p/prof -name "*kernel_stats.csv" | head -3
exit $rc
