"""AllegroKuka state dump / replay files (handarm_hip/state_files.py) on the CPU: the chunk format and the
load loop of allegro_kuka_base.py:1506-1592, and the episode recorder against a per-env-list restatement of
accumulate_env_states / dump_env_states (:1493-1543)."""
import io
import random

import pytest
import torch

from handarm_hip import state_files as SF


def _decode(data):
    """Split a dump into (count, root, dof) chunks by the byte format (u32 big-endian prefixes)."""
    f = io.BytesIO(bytes(data))
    out = []
    while True:
        h = f.read(4)
        if not h:
            return out
        k = int.from_bytes(h, "big")
        ts = []
        for _ in range(2):
            n = int.from_bytes(f.read(4), "big")
            ts.append(torch.load(io.BytesIO(f.read(n)), weights_only=True))
        out.append((k, ts[0], ts[1]))


def test_chunk_round_trip_and_last_chunk_loaded_twice(tmp_path):
    p = tmp_path / "states.bin"
    r1, d1 = torch.randn(2, 4, 13), torch.randn(2, 23, 2)
    r2, d2 = torch.randn(3, 4, 13), torch.randn(3, 23, 2)
    SF.append_chunks(p, [SF.encode_chunk(r1, d1)])
    SF.append_chunks(p, [SF.encode_chunk(r2, d2)])
    SF.append_chunks(p, [])                                     # nothing to write: file unchanged
    ch = _decode(p.read_bytes())
    assert [c[0] for c in ch] == [2, 3]
    root, dof = SF.read_state_file(p)
    # the reference's finally-clause parse re-appends the last chunk at the end of the file
    assert torch.equal(root, torch.cat([r1, r2, r2]))
    assert torch.equal(dof, torch.cat([d1, d2, d2]))


def test_empty_or_truncated_file(tmp_path):
    p = tmp_path / "empty.bin"
    p.write_bytes(b"")
    with pytest.raises(RuntimeError):
        SF.read_state_file(p)
    q = tmp_path / "trunc.bin"
    r, d = torch.randn(2, 4, 13), torch.randn(2, 23, 2)
    q.write_bytes(bytes(SF.encode_chunk(r, d)) + b"\x00\x00\x00\x05\x00\x00")   # a second chunk cut short
    root, dof = SF.read_state_file(q)
    assert torch.equal(root, torch.cat([r, r])) and torch.equal(dof, torch.cat([d, d]))


class _PerEnvLists:
    """The reference's bookkeeping, restated with its per-env lists (allegro_kuka_base.py:376-377,1493-1538)."""

    def __init__(self, n):
        self.roots = [[] for _ in range(n)]
        self.dofs = [[] for _ in range(n)]

    def accumulate(self, root, dof):
        root, dof = root.clone(), dof.clone()
        for e in range(len(self.roots)):
            self.roots[e].append(root[e])
            self.dofs[e].append(dof[e])

    def dump(self, env_ids):
        out = []
        for e in env_ids:
            ep_len = len(self.roots[e])
            if ep_len <= 20:
                continue
            k = min(ep_len // 10, 50)
            idx = random.sample(range(ep_len), k)
            out.append((k, torch.stack([self.roots[e][i] for i in idx]), torch.stack([self.dofs[e][i] for i in idx])))
            self.roots[e], self.dofs[e] = [], []
        return out


def test_recorder_matches_per_env_lists():
    n, A, D = 5, 4, 23
    rec, ref = SF.EpisodeStateRecorder(n), _PerEnvLists(n)
    gen = torch.Generator().manual_seed(3)
    # a schedule with long episodes, short ones (<= 20, kept and extended), and >500-step ones (k capped at 50)
    schedule = {25: [0, 2], 31: [1], 40: [0], 52: [0, 3, 4], 70: [2], 600: [1, 2, 3], 640: [0, 1, 2, 3, 4]}
    for step in range(1, 641):
        root, dof = torch.randn(n, A, 13, generator=gen), torch.randn(n, D, 2, generator=gen)
        rec.accumulate(root, dof)
        ref.accumulate(root, dof)
        if step in schedule:
            s = random.getstate()
            got = [_decode(c)[0] for c in rec.dump(schedule[step])]
            random.setstate(s)
            want = ref.dump(schedule[step])
            assert len(got) == len(want)
            for g, w in zip(got, want):
                assert g[0] == w[0]
                assert torch.equal(g[1], w[1]) and torch.equal(g[2], w[2])
    # snapshots no env still needs are released
    assert rec.base + len(rec.hist) == 640
    assert rec.base == min(rec.start)
