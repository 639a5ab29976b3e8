set -o pipefail
mkdir -p gpurun_out/r06m
timeout -k 10 300 python -u tools/eval_ab.py tools/ablibs/libreidmi_ev256.so,tools/ablibs/libreidmi_ev128.so 3 > gpurun_out/r06m/eval_ab.txt 2>&1
rc=$?; echo "eval_ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06m/eval_ab.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for a in "ev128st market1501" "ev128st market1501 clustered" "ev128st msmt17"; do
  set -- $a
  timeout -k 10 120 python -u tools/eval_stamps.py tools/ablibs/libreidmi_$1.so $2 $3 > gpurun_out/r06m/stamps.txt 2>&1
  rc=$?; echo "== $a rc=$rc"; grep -v amdgpu.ids gpurun_out/r06m/stamps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
