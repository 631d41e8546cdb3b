"""Env sharding across GPUs: one process and one sim per GPU,
rank k owning envs [k N / G, (k+1) N / G). Envs never interact (collision
groups are per env: test10_servo_vecenv.py:317,323), so stepping needs no
collective; the concatenation of the ranks' tensors in rank order is the
single-sim layout (global index = k N / G + local index, env grid placed by
global index). The one optional collective is an all-gather of an observation
tensor for a single-process trainer — over RCCL/xGMI on MI355X (backend
"nccl"), over gloo on the host.
"""
import torch
import torch.distributed as dist


def env_range(rank, world, num_envs):
    """[start, end) of rank's envs; the remainder goes to the first ranks."""
    base, rem = divmod(num_envs, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def shard_sim(sim, rank, world, num_envs):
    """Tag a freshly created sim as rank's shard: envs it creates are placed at
    their global grid cells. Returns (start, end)."""
    start, end = env_range(rank, world, num_envs)
    sim.env_offset = start
    return start, end


def all_gather_rows(t, group=None):
    """All ranks' (n_k, ...) row blocks concatenated in rank order (all ranks
    must hold equal n_k, the weak-scaling layout). One all_gather_into_tensor:
    a single collective per step, sized n_k x world."""
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo":
        # gloo (host rehearsal, or several ranks sharing one GPU): gather host copies
        parts = [torch.empty_like(t, device="cpu") for _ in range(world)]
        dist.all_gather(parts, t.detach().to("cpu").contiguous(), group=group)
        return torch.cat(parts, 0).to(t.device)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    dist.all_gather_into_tensor(out, t.contiguous(), group=group)
    return out


def backend_for(world, device_count):
    """RCCL ("nccl") when every rank has a GPU of its own; gloo otherwise (host
    rehearsal, or ranks sharing one GPU, which RCCL does not allow)."""
    return "nccl" if world > 1 and device_count >= world else "gloo"
