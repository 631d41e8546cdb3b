"""BASELINE config 4 ("servo vecenv 32768 envs sharded across 8xMI355X") on the
one GPU the box has: 8 rank processes x 4096 servo envs, started by the bench's
own launcher (launch.spawn_ranks), each stepping its shard on cuda:0 for 60
frames under the global action bank; their all-gathered root and rigid-body
tensors must equal one 32768-env sim stepped the same way, bit for bit
(global index = k N / G + local, no interaction between shards).
The ranks share the device, so the process group is gloo; RCCL (one GPU per
rank) is what the 8-GPU node runs and is not exercised here.

Also: one 32768-env step of the device against the oracle from the same state."""
import os

import numpy as np
import pytest

from isaacgym import gymapi, gymtorch
from test_isaacgym_amd import launch, scenes
import oracle

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ENVS_PER_RANK, WORLD, FRAMES = 4096, 8, 60


def _single_sim(gym, n, frames):
    sim, _ = scenes.servo_scene(gym, n)
    gym.prepare_sim(sim)
    root = gymtorch.wrap_tensor(gym.acquire_actor_root_state_tensor(sim))
    rb = gymtorch.wrap_tensor(gym.acquire_rigid_body_state_tensor(sim))
    acts = scenes.servo_actions(n, frames, "cpu", seed=11).to("cuda:0")
    gym.refresh_actor_root_state_tensor(sim)
    for f in range(frames):
        root[:, 3:10] = acts[f]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_actor_root_state_tensor(sim)
        gym.refresh_rigid_body_state_tensor(sim)
    return sim, root, rb


def test_config4_sharded_equals_single_sim(tmp_path):
    out = str(tmp_path / "config4")
    rc, codes = launch.spawn_ranks([os.path.join(HERE, "_shard_worker_gpu.py"), str(ENVS_PER_RANK), str(FRAMES),
                                    out], WORLD, timeout=400)
    assert rc == 0, codes
    g_root, g_rb = np.load(out + "_root.npy"), np.load(out + "_rb.npy")
    gym = gymapi.acquire_gym()
    n = WORLD * ENVS_PER_RANK
    sim, root, rb = _single_sim(gym, n, FRAMES)
    want_root, want_rb = root.cpu().numpy(), rb.cpu().numpy()
    gym.destroy_sim(sim)
    assert g_root.shape == (2 * n, 13) and g_rb.shape == (2 * n, 13)
    assert np.all(np.isfinite(want_rb))
    assert np.array_equal(g_root, want_root), "root max |diff| %g" % np.abs(g_root - want_root).max()
    assert np.array_equal(g_rb, want_rb), "rb max |diff| %g" % np.abs(g_rb - want_rb).max()


def test_config4_rccl_rank_equals_single_sim(tmp_path):
    """The RCCL path of the sharded job: one rank over backend "nccl" (RCCL
    allows one rank per device, and the box has one), so the all-gather of
    the root / rigid-body tensors goes through all_gather_into_tensor on the
    device (sharding.all_gather_rows' RCCL branch, what config 4 runs on the
    8-GPU node). 4096 envs, 20 frames: equal to one sim, bit for bit."""
    out = str(tmp_path / "rccl")
    n, frames = ENVS_PER_RANK, 20
    rc, codes = launch.spawn_ranks([os.path.join(HERE, "_shard_worker_gpu.py"), str(n), str(frames), out, "nccl"],
                                   1, timeout=300)
    assert rc == 0, codes
    g_root, g_rb = np.load(out + "_root.npy"), np.load(out + "_rb.npy")
    gym = gymapi.acquire_gym()
    sim, root, rb = _single_sim(gym, n, frames)
    want_root, want_rb = root.cpu().numpy(), rb.cpu().numpy()
    gym.destroy_sim(sim)
    assert np.array_equal(g_root, want_root) and np.array_equal(g_rb, want_rb)


def test_config4_single_sim_step_matches_oracle():
    """32768 envs (65536 bodies, 1024 waves of k_rigid_step1): 5 frames of
    random teleports from the initial state, the oracle stepping alongside (its
    ground patches kept from step to step like the device's), bit for bit every
    frame — state and net contact force."""
    gym = gymapi.acquire_gym()
    n = WORLD * ENVS_PER_RANK
    sim, root, rb = _single_sim(gym, n, 0)
    ncf = gymtorch.wrap_tensor(gym.acquire_net_contact_force_tensor(sim))
    acts = scenes.servo_actions(n, 5, "cuda:0", seed=12)
    p, m = sim.mg_params(), sim.mg_model()
    cc = oracle.contact_cache(m)
    st = sim.model_arrays["body_state0"].copy()
    roots = sim.model_arrays["actor_root_body"]
    for k in range(5):
        root[:, 3:10] = acts[k]
        assert gym.set_actor_root_state_tensor(sim, gymtorch.unwrap_tensor(root))
        gym.simulate(sim)
        gym.fetch_results(sim, True)
        gym.refresh_rigid_body_state_tensor(sim)
        gym.refresh_net_contact_force_tensor(sim)
        gym.refresh_actor_root_state_tensor(sim)
        st[roots, 3:10] = acts[k].cpu().numpy()
        cf = oracle.step(p, m, st, np.zeros((0, 2), np.float32), contact_cache=cc)
        got = rb.cpu().numpy()
        assert np.array_equal(got, st), "frame %d: max |diff| %g" % (k, np.abs(got - st).max())
        assert np.array_equal(ncf.cpu().numpy(), cf), "frame %d: contact force" % k
    gym.destroy_sim(sim)
