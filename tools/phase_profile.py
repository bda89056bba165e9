"""Per-phase cycle shares of one substep (diagnostic build libhandarm_hip_prof.so, -DHA_PROFILE).

Build: hipcc ... -DHA_PROFILE -o handarm_hip/libhandarm_hip_prof.so ; run on the GPU box.
Shares are meaningful, absolute lengths are not (the stamps add barriers)."""
import ctypes as C
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "isaacgym-hand-arm_amd")]
from handarm_hip import _lib, build  # noqa: E402

PROF_LIB = os.path.join(build.PKG, os.environ.get("HA_PROF_LIB", "libhandarm_hip_prof.so"))   # A/B: another name
ENVT_LIB = os.path.join(build.PKG, os.environ.get("HA_ENVT_LIB", "libhandarm_hip_envt.so"))     # -DHA_ENVT: workgroup spans only (no phase atomics)
PHASES = ["fk", "dynamics(CRBA+RNEA)", "chol+Minv+free+objects", "detect", "contact rows J,Y", "joint rows", "PGS",
          "forces+integrate"]

if __name__ == "__main__":
    if "--build" in sys.argv:
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *build.FLAGS, *sys.argv[sys.argv.index("--build") + 1:], "-DHA_PROFILE", "-I", build.INCLUDE,
               "-o", PROF_LIB, os.path.join(build.CSRC, "handarm_hip.hip")]
        subprocess.check_call(cmd)
        subprocess.check_call([x if x != "-DHA_PROFILE" else "-DHA_ENVT" for x in cmd[:-3]] + ["-o", ENVT_LIB, cmd[-1]])
        sys.exit(0)
    envt_only = "--envt-only" in sys.argv
    _lib.LIB_PATH = ENVT_LIB if envt_only else PROF_LIB
    import torch
    from tools.perf_probe import run
    lib = _lib.load()
    if not envt_only:
        lib.ha_profile_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    raw = (C.c_ulonglong * 192)()     # two sets of 96: light substeps, then heavy ones (HA_PROFILE_HEAVY)
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    n = int(args[0]) if args else 8192

    def report(label):
        torch.cuda.synchronize()
        lib.ha_profile_read(raw, 1)
        both = [raw[i] + raw[96 + i] for i in range(96)]
        report_set(label, both)
        heavy = [raw[96 + i] for i in range(96)]
        if heavy[9]:
            print(f"  heavy substeps only (> 24 contacts offered): {100.0 * heavy[9] / max(both[9], 1):.2f}% of substeps, "
                  f"{100.0 * sum(heavy[:8]) / max(sum(both[:8]), 1):.1f}% of cycles", flush=True)
            report_set(label + " [heavy]", heavy)

    def report_set(label, buf):
        tot = sum(buf[:8])
        print(f"{label}: contacts/substep {buf[8] / max(buf[9], 1):.2f}", flush=True)
        print("  " + "  ".join(f"{PHASES[i]} {100.0 * buf[i] / tot:5.1f}%" for i in range(8)), flush=True)
        sub = max(buf[9], 1)
        for k, name in enumerate(["obj-ground", "obj-static", "obj-obj", "link-obj", "link-static", "link-link"]):
            t_, n_, h_ = (10 + k, 15 + k, 20 + k) if k < 5 else (80, 81, 82)       # self pairs (kind 5) at 80..82
            print(f"    narrow {name:10s}: {buf[n_] / sub:6.2f} pairs/substep, {buf[h_] / sub:6.2f} with contacts, "
                  f"{100.0 * buf[t_] / tot:5.1f}% of substep cycles", flush=True)
        if buf[94]:
            print(f"    broad phase: {buf[94] / sub:6.2f} batches of 64 pairs/substep (tests, record validity, face-record "
                  f"loads) {100.0 * buf[93] / tot:5.1f}% of substep cycles", flush=True)
        if buf[90]:
            print(f"    pair face records: {buf[91] / sub:6.2f} checks/substep, {buf[92] / sub:6.2f} pairs skipped; checks "
                  f"{100.0 * buf[90] / tot:5.1f}% of substep cycles", flush=True)
        if buf[88]:
            print(f"    persistent manifolds: {buf[89] / sub:6.2f} pairs/substep refreshed from their record; record checks + "
                  f"refreshes {100.0 * buf[88] / tot:5.1f}% of substep cycles", flush=True)
        if buf[85]:
            print(f"    self pass: box table + box tests {100.0 * buf[83] / tot:5.1f}%, {buf[85] / sub:6.2f} candidates/substep, "
                  f"{buf[86] / sub:6.2f} with a record, {buf[87] / sub:6.2f} skipped by it; record checks "
                  f"{100.0 * buf[84] / tot:5.1f}%", flush=True)
        print("    hull-hull split: " + "  ".join(f"{nm} {100.0 * buf[25 + i] / tot:5.1f}%" for i, nm in
              enumerate(["setup", "SAT A", "SAT B", "incident", "emit", "edge-edge", "clip"])), flush=True)
        for k, name in enumerate(["obj-ground", "obj-static", "obj-obj", "link-obj", "link-static", "link-link"]):
            row = [buf[32 + 8 * k + i] for i in range(7)]
            if sum(row):
                print(f"      {name:11s}: " + "  ".join(f"{nm} {100.0 * v / tot:5.1f}%" for nm, v in
                      zip(["setup", "SAT A", "SAT B", "incident", "emit", "edge-edge", "clip"], row)), flush=True)

    if any(f in sys.argv for f in ("--bench-scene", "--kuka", "--bin", "--allegro", "--c4")):
        # the bench workload: VecTask after its first (reset) steps, random actions
        from handarm_hip.tasks import AllegroHand, AllegroKuka, Ur5SihMultiObjectManipulation
        if "--allegro" in sys.argv:
            n = int(args[0]) if args else 16384
            env = AllegroHand({"env": {"numEnvs": n}, "seed": 42}, "cuda:0", "cuda:0")
        elif "--kuka" in sys.argv:
            n = int(args[0]) if args else 4096
            env = AllegroKuka({"env": {"numEnvs": n}, "seed": 42}, "cuda:0", "cuda:0")
        elif "--bin" in sys.argv:       # bench --task binpick (config 5 shard)
            from handarm_hip import model as HM
            pool = HM.POOL_WIDE if "--wide" in sys.argv else HM.POOL16
            env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42, "bin": {"asset": "hard_bin"},
                                                 "objects": {"num_objects": 8, "dataset": {"ycb": pool}}},
                                                "cuda:0", "cuda:0")
        elif "--c4" in sys.argv:        # bench config 4: 16-object YCB pool, DR on (--nomug: the pool without the mug)
            from handarm_hip import model as HM
            pool = HM.POOL_WIDE if "--wide" in sys.argv else HM.POOL16
            if "--nomug" in sys.argv:
                pool = [p for p in pool if "mug" not in p]
            env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42, "task": {"randomize": True},
                                                 "objects": {"dataset": {"ycb": pool}}}, "cuda:0", "cuda:0")
        else:
            env = Ur5SihMultiObjectManipulation({"env": {"numEnvs": n}, "seed": 42}, "cuda:0", "cuda:0")
        env.reset()
        na = env.num_acts
        g = torch.Generator(device="cuda:0").manual_seed(42)
        warm = int(os.environ.get("HA_PROFILE_WARM", 20))     # steps before the profiled window (episode: 200)
        # HA_PROFILE_POOL=1: bench.py's actions, a pool of 16 random action batches cycled (their mean drifts the arm)
        apool = ([torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1 for _ in range(16)]
                 if os.environ.get("HA_PROFILE_POOL") == "1" else None)
        _k = [0]

        def next_actions():
            _k[0] += 1
            return apool[_k[0] % 16] if apool else torch.rand((n, na), device="cuda:0", generator=g) * 2 - 1
        for _ in range(warm):
            env.step(next_actions())
        torch.cuda.synchronize()
        if not envt_only:
            lib.ha_profile_read(raw, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            env.step(next_actions())
        e1.record()
        torch.cuda.synchronize()
        print(f"bench scene n={n}: {e0.elapsed_time(e1) / 10:.3f} ms/step "
              f"({'workgroup-span build' if envt_only else 'profiled build'})", flush=True)
        if not envt_only:
            report("bench scene")
        if "--envt" in sys.argv or envt_only:
            # per-workgroup spans of one more step (s_memrealtime, 100 MHz): the spread of env durations, and what
            # the slow envs have in common (contacts offered, resets)
            import numpy as np
            sim = env.sim
            rb = sim.t["reset_buf"].cpu().numpy().astype(bool)
            cs0 = sim.t["contact_stats"].cpu().numpy().astype(np.int64).copy()
            env.step(next_actions())
            torch.cuda.synchronize()
            cs1 = sim.t["contact_stats"].cpu().numpy().astype(np.int64)
            cs = cs1 - cs0
            cs[:, 2] = cs1[:, 2]            # column 2 is a running maximum, not a sum
            lib.ha_profile_env_times.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
            tb = (C.c_ulonglong * (2 * n))()
            lib.ha_profile_env_times(tb, n)
            t = np.frombuffer(tb, dtype=np.uint64).reshape(n, 2).astype(np.int64)
            # the stamps are per launch slot; slot i ran env order[i] (ha_set_env_order): per env from here on
            order = sim._env_order.cpu().numpy() if getattr(sim, "rebalance_every", 0) > 0 else np.arange(n)
            t_env = np.empty_like(t)
            t_env[order] = t
            t = t_env
            hw = None
            if hasattr(lib, "ha_profile_env_hw"):
                hb = (C.c_uint * (2 * n))()
                lib.ha_profile_env_hw.argtypes = [C.POINTER(C.c_uint), C.c_int]
                lib.ha_profile_env_hw(hb, n)
                hw = np.frombuffer(hb, dtype=np.uint32).reshape(n, 2).copy()
                hw_env = np.empty_like(hw)
                hw_env[order] = hw
                hw = hw_env
            t0 = t[:, 0].min()
            dur = (t[:, 1] - t[:, 0]) * 0.01          # us
            st = (t[:, 0] - t0) * 0.01
            end = (t[:, 1] - t0) * 0.01
            print(f"env spans (us): kernel {end.max():.1f}; start p50 {np.percentile(st, 50):.1f} p99 {np.percentile(st, 99):.1f} "
                  f"max {st.max():.1f}; duration min {dur.min():.1f} p10 {np.percentile(dur, 10):.1f} "
                  f"p50 {np.percentile(dur, 50):.1f} p90 {np.percentile(dur, 90):.1f} p99 {np.percentile(dur, 99):.1f} "
                  f"max {dur.max():.1f}; mean/max {dur.mean() / dur.max():.2f}", flush=True)
            off = cs[:, 3] / np.maximum(cs[:, 0], 1)
            for lo, hi in ((0, 50), (50, 90), (90, 99), (99, 100)):
                a, b = np.percentile(dur, lo), np.percentile(dur, hi)
                sel = (dur >= a) & (dur <= b)
                print(f"  duration p{lo}-p{hi} ({a:.0f}-{b:.0f} us): {sel.sum()} envs, resets {rb[sel].mean():.3f}, "
                      f"contacts offered/substep {off[sel].mean():.2f}, mean of the env max offered (run) {cs[sel, 2].mean():.1f}, "
                      f"over capacity {cs[sel, 1].sum() / max(cs[sel, 0].sum(), 1):.4f}", flush=True)
            print(f"  corr(duration, contacts offered/substep) {np.corrcoef(dur, off)[0, 1]:.3f}, "
                  f"corr(duration, env max offered) {np.corrcoef(dur, cs[:, 2])[0, 1]:.3f}", flush=True)
            if hw is not None:
                # HW_ID: SIMD [5:4], CU [11:8], SH [12], SE [15:13]; XCC_ID [3:0]
                h0, xcc = hw[:, 0], hw[:, 1] & 15
                simd, cu, sh, se = (h0 >> 4) & 3, (h0 >> 8) & 15, (h0 >> 12) & 1, (h0 >> 13) & 7
                cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
                simd_key = cu_key * 4 + simd
                for name, key in (("CU", cu_key), ("SIMD", simd_key)):
                    u, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
                    tot = np.bincount(inv, weights=dur)
                    mx = np.zeros(len(u)); np.maximum.at(mx, inv, dur)
                    print(f"  per {name}: {len(u)} used, envs each min {cnt.min()} max {cnt.max()}; summed env time "
                          f"min {tot.min():.0f} p50 {np.median(tot):.0f} max {tot.max():.0f} us; slowest env per {name} "
                          f"min {mx.min():.0f} p50 {np.median(mx):.0f} max {mx.max():.0f} us", flush=True)
                    top = np.argsort(dur)[-max(n // 100, 1):]
                    print(f"    the 1% slowest envs: their {name}'s summed env time p50 {np.median(tot[inv[top]]):.0f} us "
                          f"(all: {np.median(tot[inv]):.0f})", flush=True)
                xs = np.unique(xcc)
                print("  per XCC: " + "  ".join(f"{x}: p50 {np.median(dur[xcc == x]):.0f} max {dur[xcc == x].max():.0f}"
                                                for x in xs), flush=True)
            hist, edges = np.histogram(dur, bins=12)
            print("  histogram: " + "  ".join(f"{edges[i]:.0f}:{hist[i]}" for i in range(12)), flush=True)
            # the slowest envs: contact_stats of the step (substeps, over capacity, max offered, offered, self,
            # refreshed records, narrow phases) and their objects (pool ids, positions)
            oid = sim.t["object_indices"].cpu().numpy() if "object_indices" in sim.t else None
            rs = sim.t["root_state"].cpu().numpy().reshape(n, -1, 13)
            for e in np.argsort(dur)[::-1][:6]:
                print(f"  slow env {e}: {dur[e]:.0f} us, start {st[e]:.0f}, stats {cs[e].tolist()}", flush=True)
                if oid is not None:
                    names = globals().get("pool")
                    ids = [names[i] if names else i for i in oid[e].tolist()]
                    print(f"    objects {ids}; actor root z {np.round(rs[e, :, 2], 3).tolist()}", flush=True)
            if os.environ.get("HA_DUMP_SLOW"):
                # the slowest envs' state after the step (every per-env tensor), for an oracle replay on the CPU
                top = np.argsort(dur)[::-1][:4]
                dump = {"envs": top, "dur": dur[top], "stats": cs[top]}
                for k, v in sim.t.items():
                    if hasattr(v, "dim") and v.dim() >= 1 and v.shape[0] >= n and v.shape[0] % n == 0:
                        vv = v.reshape(n, v.shape[0] // n, *v.shape[1:])      # (N * A, 13) rows: per env
                        dump[k] = vv[torch.as_tensor(top.copy(), device=v.device)].cpu().numpy()
                np.savez(os.environ["HA_DUMP_SLOW"], **dump)
        sys.exit(0)
    for objects in (False, True):
        lib.ha_profile_read(raw, 1)
        run(n, "objects on" if objects else "objects off", objects=objects)
        report("objects on" if objects else "objects off")
