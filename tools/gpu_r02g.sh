set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
A="timeout -k 10 120 python tools/abtest.py"
for rep in 1 2; do
for v in base seg4w8 seg4w16; do
  L=""; [ $v != base ] && L="--lib exp/liblbk8s_$v.so"
  $A $L --steps 300 > gpurun_out/abr_${v}_1m_$rep.log 2>&1 || exit 1
  $A $L --steps 300 --envs 131072 > gpurun_out/abr_${v}_131k_$rep.log 2>&1 || exit 1
done
done
timeout -k 10 200 python tools/train_bench.py > gpurun_out/train_bench_r02g.log 2>&1
rc=$?
for f in gpurun_out/abr_*.log; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f)"; done
cat gpurun_out/train_bench_r02g.log | grep "^{"
exit $rc
