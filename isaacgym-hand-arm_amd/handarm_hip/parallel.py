"""Multi-GPU: envs are sharded one process per GPU; the only cross-rank traffic is the episode-stat
reduction at log intervals. The reference logs each rank's stats separately
(rlgames_utils.py:183-219); reducing the COUNTS before the EWMA update (multi_object_manipulation.py:
324-351) gives every rank the global success rate, identical to a single-GPU run over all envs.
"""
import torch


def world():
    import torch.distributed as dist
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def reduce_episode_stats(env):
    """All-reduce (sum) the pending per-step device counters of `env` across ranks, in place.

    Payload: pending_steps x (2 + 2*pool) int32 + pending_steps x 4 float32 (a few KB); one collective
    per log interval, launched on the current stream (RCCL over xGMI with the nccl backend, gloo on CPU).
    """
    if world() == 1:
        return
    import torch.distributed as dist
    k = env._stat_pending
    if k == 0:
        return
    R = env.sim.stats_ring
    slots = torch.tensor([(env._stat_folded + s) % R for s in range(k)], device=env.sim.t["stats"].device)
    stats = env.sim.t["stats"].index_select(0, slots)
    terms = env.sim.t["term_sums"].index_select(0, slots)
    dist.all_reduce(stats)
    dist.all_reduce(terms)
    env.sim.t["stats"].index_copy_(0, slots, stats)
    env.sim.t["term_sums"].index_copy_(0, slots, terms)
    env.stat_scale = world()          # EWMA alpha uses the GLOBAL number of envs


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


def fold_counts(stats, terms, num_envs, ewma, obj_ewma, object_names):
    """Host EWMA update from (already reduced) per-step counters; mirrors _update_success_rate and the
    reward-term logging (multi_object_manipulation.py:305-351).

    stats: (steps, 2 + 2*n_obj) ints [resets, successes, (resets_i, successes_i)...];
    terms: (steps, 4) float reward-term sums; num_envs: GLOBAL env count.
    Returns (log dict, ewma, obj_ewma, resets, successes)."""
    import numpy as np
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


__all__ = ["reduce_episode_stats", "reduce_kuka_episode_stats", "fold_counts", "world"]
_ = torch
