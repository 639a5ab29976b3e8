set -o pipefail
mkdir -p gpurun_out/r06aa
timeout -k 10 300 python -u tools/eval_ab.py tools/ablibs/libreidmi_evm0.so,tools/ablibs/libreidmi_evm1.so 3 > gpurun_out/r06aa/eval_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06aa/eval_ab.txt | grep "^r[12]"
exit $rc
