"""Multi-GPU: envs are sharded one process per GPU; the only cross-rank traffic is the episode-stat
reduction at log intervals. The reference logs each rank's stats separately
(rlgames_utils.py:183-219); reducing the COUNTS before the EWMA update (multi_object_manipulation.py:
324-351) gives every rank the global success rate, identical to a single-GPU run over all envs.

Process model (utils/rlgames_utils.py:85-107, utils/utils.py:94): one process per GPU, launched by
torchrun; RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* come from the environment, the sim device is
cuda:LOCAL_RANK and the seed is seed + rank. ``init_distributed`` is that bring-up (bench.py and any
training driver call it); the backend is "nccl" (RCCL over xGMI on ROCm) for GPU ranks and "gloo" on CPU.
"""
import os

import numpy as np
import torch


def world():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank():
    import torch.distributed as dist
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_distributed(backend=None):
    """One process per GPU from torchrun's environment. Returns (rank, local_rank, world_size, device).

    world_size 1 (no WORLD_SIZE, or 1): no process group, device cuda:0 (cpu with backend "gloo").
    world_size > 1: init_process_group(backend) over MASTER_ADDR (default 127.0.0.1) / MASTER_PORT; "nccl"
    binds the group to cuda:LOCAL_RANK."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rk = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal on a box with fewer GPUs than ranks: HA_DIST_BACKEND=gloo HA_DIST_SHARE_GPU=1 puts rank r on
    # cuda:(r % device_count) and reduces over gloo (RCCL needs one GPU per rank)
    backend = os.environ.get("HA_DIST_BACKEND", backend or "nccl")
    if backend == "nccl":
        device = f"cuda:{lr}"
    elif os.environ.get("HA_DIST_SHARE_GPU") == "1" and torch.cuda.is_available():
        device = f"cuda:{lr % torch.cuda.device_count()}"
    else:
        device = "cpu"
    if device != "cpu":
        torch.cuda.set_device(device)
    if ws > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": torch.device(device)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rk, world_size=ws, **kw)
    return rk, lr, ws, device


def describe():
    """The process group as bench.py reports it: backend and the world size an all-reduce of ones over it counts
    (so a scaling record shows that RCCL saw every rank). No process group: backend None."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return {"backend": None, "world_size": 1}
    dev = f"cuda:{torch.cuda.current_device()}" if dist.get_backend() == "nccl" else "cpu"
    t = torch.ones(1, device=dev)
    dist.all_reduce(t)
    return {"backend": dist.get_backend(), "world_size": int(t.item())}


def global_num_envs(env):
    """Number of envs over ALL ranks (the EWMA's alpha divides by it). Shards may differ in size, so it is
    all-reduced once (the first multi-rank fold, on every rank) and cached on the env."""
    n = getattr(env, "_global_num_envs", None)
    if n is None:
        n = env.num_envs
        if world() > 1:
            import torch.distributed as dist
            t = torch.tensor([n], dtype=torch.int64, device=env.sim.t["stats"].device)
            dist.all_reduce(t)
            n = int(t.item())
        env._global_num_envs = n
    return n


def pending_slots(env):
    R = env.sim.stats_ring
    return [(env._stat_folded + s) % R for s in range(env._stat_pending)]


def fold_pending(env, num_envs):
    """Fold the pending device ring slots of `env` into its EWMA state and log dict, then mark them folded.
    num_envs: the env count the counters cover (global after a cross-rank reduce)."""
    slots = pending_slots(env)
    if not slots:
        return
    stats = env.sim.t["stats"].cpu().numpy()[slots]
    terms = env.sim.t["term_sums"].cpu().numpy()[slots]
    env._stat_pending = 0
    env._stat_folded += len(slots)
    log, env._success_rate_ewma, env._object_ewma, r, sc = fold_counts(
        stats, terms, num_envs, env._success_rate_ewma, env._object_ewma, env.objects)
    env._log_data.update(log)
    env.total_num_resets += r
    env.total_num_successes += sc


def reduce_episode_stats(env):
    """All-reduce (sum) the pending per-step device counters of `env` across ranks, then fold them at the
    global env count. Every ring slot is reduced exactly once: the fold marks it done, so a later call (or
    the ring-full fold in step()) only sees new slots. A collective: every rank calls it at the same step
    (bench.py's log interval; the task's step() when the ring is full).

    Payload: pending_steps x (2 + 2*pool) int32 + pending_steps x 4 float32 (a few KB); one collective
    per log interval, launched on the current stream (RCCL over xGMI with the nccl backend, gloo on CPU).
    Single rank: a plain local fold."""
    if world() == 1:
        fold_pending(env, env.num_envs)
        return
    import torch.distributed as dist
    n = global_num_envs(env)
    if env._stat_pending:
        slots = torch.tensor(pending_slots(env), device=env.sim.t["stats"].device)
        stats = env.sim.t["stats"].index_select(0, slots)
        terms = env.sim.t["term_sums"].index_select(0, slots)
        dist.all_reduce(stats)
        dist.all_reduce(terms)
        env.sim.t["stats"].index_copy_(0, slots, stats)
        env.sim.t["term_sums"].index_copy_(0, slots, terms)
    fold_pending(env, n)


def reduce_kuka_episode_stats(env):
    """AllegroKuka: global means of the logged per-env scalars (prev_episode_successes, true_objective) over
    all ranks' envs. One all-reduce of a 3-float payload (sums and env count) per log interval; returns
    {"successes": .., "true_objective_mean": ..} as device tensors (no host sync)."""
    ts = env.task_state
    from . import model as HM
    v = torch.full((3,), float(ts.shape[0]), device=ts.device)       # device fill: no host->device copy/sync
    v[0:2] = ts[:, HM.AK_PREV_SUCC:HM.AK_TRUE_OBJ + 1].sum(0)        # adjacent fields (8, 9): a slice, no index copy
    if world() > 1:
        import torch.distributed as dist
        dist.all_reduce(v)
    return {"successes": v[0] / v[2], "true_objective_mean": v[1] / v[2]}


def reduce_allegro_episode_stats(env):
    """AllegroHand: consecutive_successes is a per-shard EWMA of the mean successes of the reset envs
    (allegro_hand.py:700-705); the global view is the env-weighted mean over ranks. One all-reduce of 2 floats;
    returns {"consecutive_successes": ..} as a device tensor."""
    cs = env.consecutive_successes.reshape(()).float()
    v = torch.full((2,), float(env.num_envs), device=cs.device)    # device fill: no host tensor per call
    v[0] = v[0] * cs
    if world() > 1:
        import torch.distributed as dist
        dist.all_reduce(v)
    return {"consecutive_successes": v[0] / v[1]}


def fold_counts(stats, terms, num_envs, ewma, obj_ewma, object_names):
    """Host EWMA update from (already reduced) per-step counters; mirrors _update_success_rate and the
    reward-term logging (multi_object_manipulation.py:305-351).

    stats: (steps, 2 + 2*n_obj) ints [resets, successes, (resets_i, successes_i)...];
    terms: (steps, 4) float reward-term sums; num_envs: GLOBAL env count.
    Returns (log dict, ewma, obj_ewma, resets, successes)."""
    F = np.float32
    log, obj_ewma = {}, list(obj_ewma)
    n_obj = len(object_names)
    total_r = total_s = 0
    for st, ts in zip(stats, terms):
        for j, name in enumerate(("reaching", "lifting", "goal", "success")):
            log["reward_terms/" + name] = float(F(ts[j]) / F(num_envs))
        r, s = int(st[0]), int(st[1])
        if r > 0:
            alpha = F(0.2) * (F(r) / F(num_envs))
            ewma = float(alpha * (F(s) / F(r)) + (F(1) - alpha) * F(ewma))
            log["success_rate_ewma/overall"] = ewma
            total_r += r
            total_s += s
        for i in range(n_obj):
            ri, si = int(st[2 + 2 * i]), int(st[3 + 2 * i])
            if ri > 0:
                alpha = F(0.2) * (F(ri) / F(num_envs)) * F(n_obj)
                obj_ewma[i] = float(alpha * (F(si) / F(ri)) + (F(1) - alpha) * F(obj_ewma[i]))
                log["success_rate_ewma/" + object_names[i]] = obj_ewma[i]
    return log, ewma, obj_ewma, total_r, total_s


__all__ = ["init_distributed", "describe", "global_num_envs", "reduce_episode_stats", "reduce_kuka_episode_stats",
           "reduce_allegro_episode_stats", "fold_counts", "fold_pending", "world", "rank"]
