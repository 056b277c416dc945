set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r02e.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_131k_tpe -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --envs 131072 > gpurun_out/prof_131k_tpe.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_131k_slice -o run --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --envs 131072 --geometry slice > gpurun_out/prof_131k_slice.log 2>&1
rc=$?
tail -n 3 gpurun_out/pytest_gpu_r02e.log
for d in prof_131k_tpe prof_131k_slice; do echo $d; grep -h "k_step\|k_reset" gpurun_out/$d/run_kernel_stats.csv | cut -d, -f1-7; done
exit $rc
