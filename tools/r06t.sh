set -o pipefail
mkdir -p gpurun_out/r06t
timeout -k 10 500 python -u tools/walk_ab.py 3 --shapes proj,out --walks 1,-3 > gpurun_out/r06t/walk_ab.txt 2>&1
rc=$?; echo "walk rc=$rc"; grep -v amdgpu.ids gpurun_out/r06t/walk_ab.txt
exit $rc
