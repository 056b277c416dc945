set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 120 python tools/abtest.py"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02d.log 2>&1 && \
$A --steps 300 > gpurun_out/ab1_base_1m.log 2>&1 && \
$A --lib exp/liblbk8s_w5.so --steps 300 > gpurun_out/ab1_w5_1m.log 2>&1 && \
$A --steps 300 > gpurun_out/ab2_base_1m.log 2>&1 && \
$A --lib exp/liblbk8s_w5.so --steps 300 > gpurun_out/ab2_w5_1m.log 2>&1 && \
$A --steps 300 --lockstep > gpurun_out/ab_base_1m_lock.log 2>&1 && \
$A --steps 300 --envs 131072 > gpurun_out/ab_base_131k.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02d -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r02d.log 2>&1
rc=$?
tail -n 2 gpurun_out/pytest_gpu_r02d.log
for f in gpurun_out/ab*_*.log; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*' $f) $(grep -o '"frac": [0-9.]*' $f)"; done
grep -h "k_step_tpe\|k_reset_listed" gpurun_out/prof_r02d/run_kernel_stats.csv | cut -d, -f1-7
exit $rc
