set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 200 python -u tools/rowread_bw.py > gpurun_out/r06n/rowread.txt 2>&1
rc=$?; echo "rowread rc=$rc"; grep -v amdgpu.ids gpurun_out/r06n/rowread.txt
exit $rc
