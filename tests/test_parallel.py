"""Multi-rank path on CPU (gloo, world size 2): the episode-stat all-reduce + EWMA fold.

SURVEY.md §8e: envs shard with no data-path collective; the only exchange is the per-log-interval
reduction of the success/reset counters, which must happen BEFORE the EWMA update
(multi_object_manipulation.py:324-351) so every rank logs the global success rate a single process over
all envs would log.
"""
import os
import socket
import types

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from handarm_hip import parallel

OBJECTS = ["015_peach", "005_tomato_soup_can", "006_mustard_bottle"]
N_LOCAL, RING = 64, 8


def local_counts(rank, k, first_slot):
    """Deterministic per-rank counters for k pending steps starting at ring slot first_slot."""
    g = np.random.default_rng(100 + rank)
    stats = np.zeros((RING, 2 + 2 * len(OBJECTS)), np.int32)
    terms = np.zeros((RING, 4), np.float32)
    for s in range(k):
        slot = (first_slot + s) % RING
        per_r = g.integers(0, 8, len(OBJECTS))
        per_s = np.minimum(per_r, g.integers(0, 8, len(OBJECTS)))
        stats[slot, 0], stats[slot, 1] = per_r.sum(), per_s.sum()
        stats[slot, 2::2], stats[slot, 3::2] = per_r, per_s
        terms[slot] = g.uniform(0, 50, 4).astype(np.float32)
    return stats, terms


def shard_envs(rank):
    return N_LOCAL + 16 * rank                      # unequal shards: the EWMA alpha needs the GLOBAL count


def fake_env(rank, k, folded):
    stats, terms = local_counts(rank, k, folded % RING)
    sim = types.SimpleNamespace(stats_ring=RING, t={"stats": torch.from_numpy(stats), "term_sums": torch.from_numpy(terms)})
    return types.SimpleNamespace(sim=sim, _stat_pending=k, _stat_folded=folded, num_envs=shard_envs(rank),
                                 objects=OBJECTS, _success_rate_ewma=0.0, _object_ewma=[0.0] * 3, _log_data={},
                                 total_num_resets=0, total_num_successes=0)


def more_counts(rank, k2, first_slot):
    """A second batch of pending steps (what the device writes between two log intervals)."""
    return local_counts(rank + 10, k2, first_slot)


def _worker(rank, world, port, k, folded, k2, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        env = fake_env(rank, k, folded)
        parallel.reduce_episode_stats(env)
        assert env._stat_pending == 0 and env._stat_folded == folded + k
        first = env.sim.t["stats"].numpy()[[(folded + s) % RING for s in range(k)]].copy()
        parallel.reduce_episode_stats(env)          # nothing pending: no slot is reduced twice
        again = env.sim.t["stats"].numpy()[[(folded + s) % RING for s in range(k)]].copy()
        st2, tm2 = more_counts(rank, k2, (folded + k) % RING)
        s2 = [(folded + k + s) % RING for s in range(k2)]
        env.sim.t["stats"][s2] = torch.from_numpy(st2[s2])
        env.sim.t["term_sums"][s2] = torch.from_numpy(tm2[s2])
        env._stat_pending = k2
        parallel.reduce_episode_stats(env)
        q.put((rank, env._global_num_envs, first.tolist(), again.tolist(), env._success_rate_ewma, env._object_ewma,
               env.total_num_resets, env.total_num_successes, sorted(env._log_data)))
    finally:
        torch.distributed.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("k,folded,k2", [(5, 0, 3), (6, 6, 4)])    # second case wraps around the ring
def test_reduce_then_fold_matches_single_process(k, folded, k2):
    """Two log intervals on unequal shards: each slot is reduced exactly once, and the EWMA after both equals
    one process folding the summed counters over all envs."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, k, folded, k2, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n_all = sum(shard_envs(r) for r in range(world))
    slots = [(folded + s) % RING for s in range(k)]
    slots2 = [(folded + k + s) % RING for s in range(k2)]
    tot_st = sum(local_counts(r, k, folded % RING)[0] for r in range(world))[slots]
    tot_tm = sum(local_counts(r, k, folded % RING)[1] for r in range(world))[slots]
    tot_st2 = sum(more_counts(r, k2, (folded + k) % RING)[0] for r in range(world))[slots2]
    tot_tm2 = sum(more_counts(r, k2, (folded + k) % RING)[1] for r in range(world))[slots2]
    ref = parallel.fold_counts(tot_st, tot_tm, n_all, 0.0, [0.0] * 3, OBJECTS)
    ref2 = parallel.fold_counts(tot_st2, tot_tm2, n_all, ref[1], ref[2], OBJECTS)
    for rank, n_glob, first, again, ewma, obj, r, s, keys in out:
        assert n_glob == n_all
        np.testing.assert_array_equal(np.array(first), tot_st)
        np.testing.assert_array_equal(np.array(again), tot_st)        # the empty second reduce changed nothing
        assert ewma == pytest.approx(ref2[1], rel=1e-6) and obj == pytest.approx(ref2[2], rel=1e-6)
        assert (r, s) == (ref[3] + ref2[3], ref[4] + ref2[4]) and r > 0
        assert set(keys) == set(ref[0]) | set(ref2[0])


def test_single_rank_folds_locally():
    env = fake_env(0, 3, 0)
    before = env.sim.t["stats"].clone()
    parallel.reduce_episode_stats(env)          # no process group: a plain local fold, counters untouched
    assert torch.equal(before, env.sim.t["stats"]) and env._stat_pending == 0 and env._stat_folded == 3
    st, tm = local_counts(0, 3, 0)
    ref = parallel.fold_counts(st[:3], tm[:3], env.num_envs, 0.0, [0.0] * 3, OBJECTS)
    assert env._success_rate_ewma == ref[1] and env.total_num_resets == ref[3]


def test_fold_counts_ewma_arithmetic():
    """Pins fold_counts to the reference update: alpha = 0.2 * resets / N (per object: x n_obj)."""
    st = np.array([[4, 1, 2, 1, 1, 0, 1, 0]], np.int32)
    tm = np.array([[1.0, 2.0, 3.0, 4.0]], np.float32)
    log, ewma, obj, r, s = parallel.fold_counts(st, tm, 8, 0.5, [0.5, 0.5, 0.5], OBJECTS)
    a = np.float32(0.2) * np.float32(4 / 8)
    assert ewma == pytest.approx(float(a * np.float32(0.25) + (1 - a) * np.float32(0.5)), rel=1e-7)
    a0 = np.float32(0.2) * np.float32(2 / 8) * 3
    assert obj[0] == pytest.approx(float(a0 * np.float32(0.5) + (1 - a0) * np.float32(0.5)), rel=1e-7)
    assert log["reward_terms/goal"] == pytest.approx(3.0 / 8)
    assert (r, s) == (4, 1)


def _kuka_worker(rank, world, port, q):
    from handarm_hip import model as HM
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7 + rank)
        ts = torch.zeros((N_LOCAL + 8 * rank, HM.AK_TS))           # ranks may hold different env counts
        ts[:, HM.AK_PREV_SUCC] = torch.randint(0, 9, (ts.shape[0],), generator=g).float()
        ts[:, HM.AK_TRUE_OBJ] = torch.rand(ts.shape[0], generator=g)
        out = parallel.reduce_kuka_episode_stats(types.SimpleNamespace(task_state=ts))
        q.put((rank, float(out["successes"]), float(out["true_objective_mean"]), ts.numpy().tolist()))
    finally:
        torch.distributed.destroy_process_group()


def test_kuka_episode_stats_are_global_means():
    """AllegroKuka: extras["successes"] / true_objective_mean after the all-reduce equal the means over the
    union of all ranks' envs (what one process over all envs reports)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_kuka_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from handarm_hip import model as HM
    allts = np.concatenate([np.array(o[3], np.float32) for o in out])
    for rank, succ, tobj, _ in out:
        np.testing.assert_allclose(succ, allts[:, HM.AK_PREV_SUCC].mean(), rtol=1e-6)
        np.testing.assert_allclose(tobj, allts[:, HM.AK_TRUE_OBJ].mean(), rtol=1e-6)


def _allegro_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = N_LOCAL + 32 * rank
        cs = torch.tensor([1.5 + rank], dtype=torch.float32)
        out = parallel.reduce_allegro_episode_stats(types.SimpleNamespace(consecutive_successes=cs, num_envs=n))
        q.put((rank, float(out["consecutive_successes"]), n, float(cs), parallel.describe()))
    finally:
        torch.distributed.destroy_process_group()


def test_allegro_episode_stats_and_group_description():
    """AllegroHand: the global consecutive_successes is the env-weighted mean of the ranks' shard EWMAs; and
    parallel.describe() (the bench line's "distributed" record) reports the backend and the world size an
    all-reduce over the group counts."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_allegro_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = sum(o[2] * o[3] for o in out) / sum(o[2] for o in out)
    for rank, got, _, _, desc in out:
        assert got == pytest.approx(want, rel=1e-6)
        assert desc == {"backend": "gloo", "world_size": 2}
    assert parallel.describe() == {"backend": None, "world_size": 1}
