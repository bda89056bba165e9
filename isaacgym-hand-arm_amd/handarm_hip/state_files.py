"""AllegroKuka state dump / replay files (cfg env.saveStates / env.loadInitialStates, AllegroKuka.yaml:90-94).

Byte format of allegro_kuka_base.py:1506-1543 / 1545-1592: the file is a sequence of chunks, one per env whose
episode was sampled,
    u32 big-endian  number of states in the chunk
    u32 big-endian  length L1, then L1 bytes: torch.save of the root states  (k, num_actors, 13)
    u32 big-endian  length L2, then L2 bytes: torch.save of the DOF states   (k, num_dofs, 2)
Chunks are appended (file mode "ab") on every reset_idx. Actor rows follow the reference's per-env order
(arm+hand, cube, table, goal; model.actor_object0 is the cube).

Loading uses torch.load(weights_only=True): the payloads are plain tensors, so nothing in the file is executed.
"""
import io
import random

import torch


def _tensor_bytes(t):
    buf = io.BytesIO()
    torch.save(t, buf)
    return buf.getbuffer()


def encode_chunk(root_states, dof_states):
    """One chunk (allegro_kuka_base.py:1524-1535): the state count, then the two length-prefixed tensors."""
    out = io.BytesIO()
    out.write(int(root_states.shape[0]).to_bytes(4, "big"))
    for t in (root_states, dof_states):
        b = _tensor_bytes(t)
        out.write(int(len(b)).to_bytes(4, "big"))
        out.write(b)
    return out.getbuffer()


def append_chunks(path, chunks):
    """Append encoded chunks to path; nothing is written when there are none (allegro_kuka_base.py:1540-1543)."""
    data = b"".join(bytes(c) for c in chunks)
    with open(path, "ab") as f:
        if len(data) > 0:
            print(f"Writing {len(data)} to file {path}")
            f.write(data)


def read_state_file(path, device="cpu"):
    """load_initial_states (allegro_kuka_base.py:1545-1592) -> (root_states, dof_states), concatenated over chunks.

    The reference parses each chunk in the `finally` of its read loop, so the pass that hits the end of the file
    parses the previous chunk's bytes again: the last chunk is loaded twice. This is kept, so that the loaded
    state count and the order in which resets cycle through the states are the reference's. A file without a
    single complete chunk raises (the reference fails there with an unbound-variable error)."""
    roots, dofs = [], []
    root_b = dof_b = None
    with open(path, "rb") as f:

        def read_n(n):
            b = f.read(n)
            if len(b) < n:
                raise RuntimeError(f"Could not read {n} bytes from the binary file. Perhaps reached the end of file")
            return b

        while True:
            end = False
            try:
                int.from_bytes(read_n(4), "big")
                root_b = read_n(int.from_bytes(read_n(4), "big"))
                dof_b = read_n(int.from_bytes(read_n(4), "big"))
            except RuntimeError as exc:
                print(exc)
                end = True
            if root_b is None or dof_b is None:
                raise RuntimeError(f"{path}: no complete state chunk")
            roots.append(torch.load(io.BytesIO(root_b), map_location=device, weights_only=True))
            dofs.append(torch.load(io.BytesIO(dof_b), map_location=device, weights_only=True))
            if end:
                break
    root = torch.cat(roots)
    dof = torch.cat(dofs)
    assert dof.shape[0] == root.shape[0]
    print(f"{len(root)} states loaded from file {path}!")
    return root, dof


class EpisodeStateRecorder:
    """accumulate_env_states / dump_env_states (allegro_kuka_base.py:1493-1543) without a Python loop per env and
    step: each step's root and DOF state tensors are kept once (one device clone each, as the reference's
    per-env clones), and every env remembers the step its current list starts at. Snapshots older than every
    env's start are released."""

    def __init__(self, num_envs):
        self.hist = []            # [(root (N, A, 13), dof (N, D, 2))], hist[i] is global step base + i
        self.base = 0
        self.start = [0] * num_envs

    def accumulate(self, root_state, dof_state):
        self.hist.append((root_state.clone(), dof_state.clone()))

    def dump(self, env_ids):
        """Chunks for the listed envs, in order: an env with more than 20 recorded states gives
        min(len // 10, 50) of them, picked with random.sample, and its list is cleared; shorter lists are
        kept and keep growing (allegro_kuka_base.py:1517-1538)."""
        chunks = []
        end = self.base + len(self.hist)
        for env in env_ids:
            env = int(env)
            b = self.start[env]
            ep_len = end - b
            if ep_len <= 20:
                continue
            k = min(ep_len // 10, 50)
            idx = random.sample(range(ep_len), k)
            print(f"Adding {k} states {idx}")
            root = torch.stack([self.hist[b + si - self.base][0][env] for si in idx])
            dof = torch.stack([self.hist[b + si - self.base][1][env] for si in idx])
            chunks.append(encode_chunk(root, dof))
            self.start[env] = end
        drop = min(self.start) - self.base
        if drop > 0:
            del self.hist[:drop]
            self.base += drop
        return chunks
