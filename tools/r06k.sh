set -o pipefail
mkdir -p gpurun_out/r06k
timeout -k 10 300 python -u tools/eval_ab.py tools/ablibs/libreidmi_evold.so,tools/ablibs/libreidmi_evnew.so,tools/ablibs/libreidmi_evpf.so 3 > gpurun_out/r06k/eval_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06k/eval_ab.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for a in "evst market1501" "evst market1501 clustered" "evpfst market1501 clustered" "evst msmt17" "evpfst msmt17"; do
  set -- $a
  timeout -k 10 120 python -u tools/eval_stamps.py tools/ablibs/libreidmi_$1.so $2 $3 > gpurun_out/r06k/stamps_$1_$2_$3.txt 2>&1
  rc=$?; echo "== $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r06k/stamps_$1_$2_$3.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
