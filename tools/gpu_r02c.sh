set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 120 python tools/abtest.py"
$A --steps 200 > gpurun_out/ab_base_1m.log 2>&1 && \
$A --lib exp/liblbk8s_w5.so --steps 200 > gpurun_out/ab_w5_1m.log 2>&1 && \
$A --steps 300 --envs 131072 > gpurun_out/ab_base_131k.log 2>&1 && \
$A --lib exp/liblbk8s_w5.so --steps 300 --envs 131072 > gpurun_out/ab_w5_131k.log 2>&1 && \
$A --steps 300 --envs 131072 --geometry slice > gpurun_out/ab_slice_131k.log 2>&1 && \
$A --steps 300 --envs 131072 --lockstep > gpurun_out/ab_base_131k_lock.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02c -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r02c.log 2>&1
rc=$?
for f in gpurun_out/ab_*.log; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"frac": [0-9.]*' $f)"; done
exit $rc
