set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lean_oracle.py tests/test_gpu_lean.py > gpurun_out/r06_lean_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06_lean_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_session.sh ab r06_ab_split128.jsonl "131072 1048576" "20,100" gym-loadbalancing_amd/lbk8s/liblbk8s.so exp/liblbk8s_split128.so || exit 1
: > gpurun_out/r06_bench_k20.jsonl
for r in 1 2; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> gpurun_out/r06_bench_k20.jsonl 2>>gpurun_out/r06_bench.err || exit 1; done
for r in 1 2; do timeout -k 10 300 python3 bench.py --weak --envs 131072 --steps 20 --warmup 5 --no-cpu-baseline --no-step-line >> gpurun_out/r06_bench_k20.jsonl 2>>gpurun_out/r06_bench.err || exit 1; done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06_bench_k20.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["envs_per_gpu"], round(r["kernel_ms"] * 1e3, 2), "us/step", f'{d["value"]:.3e}', "frac", round(r["frac"], 3), r["kernel"].split()[0])
PY
