set -o pipefail
mkdir -p gpurun_out/r06h
A=tools/ablibs
timeout -k 10 400 python -u tools/lib_ab.py $A/libreidmi_gbase.so,$A/libreidmi_gGELU1.so,$A/libreidmi_gNOGELU.so 3 --shapes cfc --M 4068291 > gpurun_out/r06h/gemm_gelu_ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/r06h/gemm_gelu_ab.txt | tail -10
if [ $rc -ne 0 ]; then exit $rc; fi
for B in 8192 19281 4096; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-msmt17 --no-rerank --no-text --no-cpu-baseline --no-backend --no-preprocess --no-jpeg --files-batch $B > gpurun_out/r06h/bench_files_$B.json 2> gpurun_out/r06h/bench_files_$B.err
  rc=$?; echo "bench $B rc=$rc"; python -c "import json,sys; d=json.loads(open('gpurun_out/r06h/bench_files_$B.json').read().strip().splitlines()[-1]); print($B, d['value'], d['files_to_map']['walls_s'], d['files_to_map']['hbm_resident_step_s'])"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
