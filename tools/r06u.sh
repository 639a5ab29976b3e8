set -o pipefail
mkdir -p gpurun_out/r06u
timeout -k 10 300 python -u tools/qkv_epi_ab.py 19281 3 > gpurun_out/r06u/qkv_epi_ab.txt 2>&1
rc=$?; echo "qkv rc=$rc"; grep -v amdgpu.ids gpurun_out/r06u/qkv_epi_ab.txt
exit $rc
