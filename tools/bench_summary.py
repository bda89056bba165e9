"""One-line-per-config summary of a bench.py JSON line (headline + configs sub-records, with the episode windows)."""
import json
import sys


def show(tag, r):
    c = r.get("contacts", {}) or {}
    line = (f"{tag}: {r['value'] / 1e6:.3f} M env-steps/s, {r['ms_per_step']:.3f} ms/step, kernel "
            f"{r['roofline']['kernel_avg_ms']:.3f} ms, HBM frac {r['roofline']['frac']:.4f}")
    if c:
        line += (f"; contacts cap {c.get('capacity')} over {c.get('at_capacity_frac', 0):.5f} mean "
                 f"{c.get('offered_mean', 0):.2f} max {c.get('offered_max')} env-max p99 {c.get('env_max_p99')}")
    print(line)
    e = r.get("episode_window")
    if e:
        c = e["contacts"]
        print(f"   episode window ({e['steps']} steps): {e['value'] / 1e6:.3f} M env-steps/s, {e['ms_per_step']:.3f} ms/step;"
              f" over {c['at_capacity_frac']:.5f} mean {c['offered_mean']:.2f} max {c['offered_max']} "
              f"env-max p99 {c['env_max_p99']}")


d = json.load(open(sys.argv[1]))
show("C2" if "configs" in d else "head", d)
for k, r in d.get("configs", {}).items():
    show(k, r)
