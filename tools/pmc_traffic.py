#!/usr/bin/env python3
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; tools/pmc_probe.py workload) into
profiles/pmc_traffic.json: HBM bytes per lb_step launch.

Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE tallies 128-B memory requests
at 64 B, i.e. reports half of a wide coalesced read stream; WRITE_SIZE is exact.  The probe
also runs 1 GiB device copies (known bytes), and the correction factor applied to the
kernel's FETCH_SIZE is measured from those (expected 2.0).

    python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
        --config default --envs 1048576 [--out profiles/pmc_traffic.json]
"""
import argparse
import csv
import json
import statistics


def per_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]) * 1024.0)  # KB -> B
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--config", default="default")
    ap.add_argument("--envs", type=int, default=1 << 20)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--steps-per-launch", type=int, default=16, help="lb_rollout launches: vector steps each")
    args = ap.parse_args()
    f = per_kernel(args.fetch_csv, "FETCH_SIZE")
    w = per_kernel(args.write_csv, "WRITE_SIZE")
    roll = [k for k in f if "k_rollout" in k]
    step = roll[0] if roll else [k for k in f if "k_step" in k][0]
    steps_per_launch = args.steps_per_launch if roll else 1
    copy = [k for k in f if "copyBuffer" in k]
    copy_bytes = float(1 << 30)
    factor = copy_bytes / statistics.median(f[copy[0]]) if copy else 2.0
    # the last launches are the timed-step workload (earlier ones: the stagger setup)
    fetch_raw = statistics.median(f[step][-(6 if roll else 13):])
    write = statistics.median(w[step][-(6 if roll else 13):])
    rs = [k for k in f if "k_reset_listed" in k]  # builds before the in-step auto-reset
    reset = None
    if rs:
        rf, rw = statistics.median(f[rs[0]][-13:]) * factor, statistics.median(w[rs[0]][-13:])
        reset = dict(kernel=rs[0], read_bytes=rf, write_bytes=rw, hbm_bytes_per_launch=rf + rw)
    res = dict(config=args.config, envs=args.envs, kernel=step,
               fetch_size_raw_bytes=fetch_raw, fetch_correction=factor,
               read_bytes=fetch_raw * factor, write_bytes=write,
               hbm_bytes_per_launch=fetch_raw * factor + write,
               steps_per_launch=steps_per_launch,
               hbm_bytes_per_env_step=(fetch_raw * factor + write) / args.envs / steps_per_launch,
               reset_kernel=reset,
               step_plus_reset_bytes_per_env_step=(fetch_raw * factor + write
                                                   + (reset["hbm_bytes_per_launch"] if reset else 0.0))
               / args.envs / steps_per_launch,
               calibration="1 GiB device copy: write = %.3f GiB, raw fetch = %.3f GiB" % (
                   statistics.median(w[copy[0]]) / copy_bytes if copy else float("nan"),
                   statistics.median(f[copy[0]]) / copy_bytes if copy else float("nan")))
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
