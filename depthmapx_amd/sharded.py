"""Multi-GPU choreography for the hot path (one process per GPU, torch.distributed over RCCL).

The units are source cells: rank r owns a contiguous x-major node range -- cut at equal modelled cost by
PointMap.shard_bounds (a source's sweep cost varies ~3x across a map: sources on open map edges see
more cells), or at equal node counts by shard_range.
Per step
  1. makeGraph for the owned sources (no communication: the cost-balanced bounds come from a sampled
     sweep whose counts are deterministic, so every rank cuts the same bounds on its own);
  2. all-gather of the run-length graph shards (ragged byte blobs, padded to the largest) so every
     rank holds the whole graph -- VGA BFS from any source can reach any node;
  3. VGA global for the rank's VGA sources (its preparation pre-passes split by contiguous node
     range, partial buffers all-reduced: Graph.set_prep_shard + prep_allreduce): fixed-size node chunks dealt round-robin over the
     ranks (vga_nodes), because the BFS cost of a source depends on where it sits in the plan;
  4. all-gather of the owned rows of the 7 float columns (allgather_rows_chunked).
Only 2 and 4 are collectives.  The helpers below take any torch.distributed backend, so the same
code is exercised with gloo on CPU tensors in tests/test_sharded_gloo.py.
"""
import torch


def _rccl(dist):
    """all_gather_into_tensor is the RCCL fast path; other backends take the list form."""
    try:
        return hasattr(dist, "all_gather_into_tensor") and dist.get_backend() == "nccl"
    except Exception:
        return False


def _gather_host(dist, t):
    """all_gather of equal-shaped tensors on a non-RCCL backend, staged through host memory (gloo
    rehearsals: its collectives on CUDA tensors are avoided); returns the concatenation on t's device.
    DMX_GLOO_DEVICE_TENSORS=1 hands gloo the device tensors instead (diagnostic of DESIGN.md section 5)."""
    import os
    if os.environ.get("DMX_GLOO_DEVICE_TENSORS") == "1":
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        return torch.cat(parts)
    parts = [torch.empty(t.shape, dtype=t.dtype) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, t.cpu())
    return torch.cat(parts).to(t.device)


def shard_range(n, rank, world):
    """Contiguous, balanced split of n units over `world` ranks."""
    return (n * rank) // world, (n * (rank + 1)) // world


def exchange_graph(pm, ctx, shard, dist, device):
    """Step 2 on device memory: every rank writes its run-length shard blob straight into its own slot of
    the padded exchange buffer, the buffer is all-gathered in place (RCCL all_gather_into_tensor over xGMI,
    the rank's slot as the input: no separate send buffer) and assembled into the whole graph.  The shard
    graph is closed once its blob is written, so the rank holds at most the exchange buffer and the
    assembled graph at once.  Returns (graph, {"blob_s", "allgather_s", "assemble_s", "bytes",
    "padded_bytes", "device_peak_bytes"}); the phases are bracketed by device synchronisations so that
    bench.py can size the exchange against replicated makeGraph, and device_peak_bytes is the most
    device memory in use (torch.cuda.mem_get_info: libdmx's allocations included) at the phase ends."""
    import time
    world, rank = dist.get_world_size(), dist.get_rank()
    cuda = device.type == "cuda"
    peak = [0]

    def sync():
        if cuda:
            torch.cuda.synchronize(device)
            free, total = torch.cuda.mem_get_info(device)
            peak[0] = max(peak[0], total - free)
    sync()
    t0 = time.perf_counter()
    n = shard.blob_size()
    sz = torch.tensor([n], dtype=torch.int64, device=device)
    if _rccl(dist):
        sizes = [torch.zeros_like(sz) for _ in range(world)]
        dist.all_gather(sizes, sz)
        sizes = [int(v.item()) for v in sizes]
    else:
        sizes = [int(v) for v in _gather_host(dist, sz).tolist()]
    mx = max(sizes)
    flat = torch.empty(world * mx, dtype=torch.uint8, device=device)
    mine = flat[rank * mx:(rank + 1) * mx]
    shard.write_blob_device(mine.data_ptr(), n)
    sync()
    if hasattr(shard, "close"):
        shard.close()   # the shard's pool and tables are in the blob now
    t1 = time.perf_counter()
    if _rccl(dist):
        dist.all_gather_into_tensor(flat, mine)
    else:
        # other backends (gloo rehearsals): gather through host tensors staged explicitly, one per rank
        flat.copy_(_gather_host(dist, mine))
    sync()
    t2 = time.perf_counter()
    del mine
    g = pm.assemble(ctx, [flat.data_ptr() + i * mx for i in range(world)], sizes)
    sync()
    t3 = time.perf_counter()
    del flat
    if cuda:
        # hand the buffer back to the device: libdmx sizes the VGA preparation (tile rows, partial-tile masks) from
        # hipMemGetInfo, which counts torch's cached blocks as used (memory budget)
        torch.cuda.empty_cache()
    return g, {"blob_s": t1 - t0, "allgather_s": t2 - t1, "assemble_s": t3 - t2, "bytes": sum(sizes),
               "padded_bytes": world * mx, "device_peak_bytes": peak[0] if cuda else None}


# a whole-graph makeGraph does the VGA preparation's symmetry scatter as it publishes the runs (DESIGN.md section 2,
# prep): +0.9 % of its time at 1000^2 (4.62 -> 4.66 s, round 4), where a shard leaves it to the preparation
FUSED_SCATTER_COST = 1.009


def choose_mk_mode(dist, device, world, mk_shard_s, exchange_s, shard_frac, sym_shard_s=0.0):
    """--mk-mode auto after a warm-up step run sharded: replicate (every rank builds the whole graph, no
    data-path collective) when building it all costs less than building the shard and exchanging it.
    The sharded step also pays the symmetry scatter in the VGA preparation (sym_shard_s, measured in the
    warm-up: the rank's share plus the all-reduces of its difference arrays), which a whole-graph build does
    inside makeGraph for FUSED_SCATTER_COST.  Times are the max over ranks so that every rank takes the same
    branch."""
    t = torch.tensor([mk_shard_s, exchange_s, shard_frac, sym_shard_s], dtype=torch.float64,
                     device=device if _rccl(dist) else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    mk, ex, frac, sym = (float(v) for v in t.tolist())
    replicate_s = mk / max(frac, 1e-9) * FUSED_SCATTER_COST
    shard_s = mk + ex + sym
    return ("replicate" if replicate_s < shard_s else "shard"), {"predicted_replicate_s": replicate_s,
                                                                 "predicted_shard_s": shard_s,
                                                                 "mk_shard_s": mk, "exchange_s": ex,
                                                                 "sym_shard_s": sym}


def device_view(ptr, count, dtype, device):
    """Zero-copy torch view of `count` int32 (dtype 0) / int64 (dtype 1) elements of device memory
    owned by libdmx (CUDA array interface; the memory stays libdmx's)."""
    class _View:
        pass
    v = _View()
    v.__cuda_array_interface__ = {"shape": (int(count),), "typestr": "<i4" if dtype == 0 else "<i8",
                                  "data": (int(ptr), False), "version": 2, "strides": None}
    return torch.as_tensor(v, device=device)


def prep_allreduce(dist, device):
    """The all-reduce callback of Graph.set_prep_shard: SUM over ranks in place (RCCL on the GPU;
    other backends reduce through a staging copy)."""
    def fn(ptr, count, dtype):
        t = device_view(ptr, count, dtype, device)
        if _rccl(dist):
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        else:
            host = t.cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM)
            t.copy_(host)
        torch.cuda.synchronize(device)
        return 0
    return fn


def vga_nodes(n, rank, world, chunk=4096):
    """Node indices of `rank`'s VGA sources: chunks c = rank, rank + world, ... of `chunk` nodes."""
    import numpy as np
    starts = np.arange(rank * chunk, n, world * chunk, dtype=np.int64)
    if len(starts) == 0:
        return np.zeros(0, dtype=np.int64)
    return np.concatenate([np.arange(b, min(b + chunk, n), dtype=np.int64) for b in starts])


def allgather_rows_chunked(full, n, dist, chunk=4096):
    """full: [n, k] tensor where this rank filled the rows vga_nodes(n, rank, world, chunk);
    afterwards every rank holds all rows (pure data movement: the values are copied, not summed)."""
    import numpy as np
    world, rank = dist.get_world_size(), dist.get_rank()
    lists = [torch.from_numpy(vga_nodes(n, r, world, chunk)) for r in range(world)]
    per = max(len(l) for l in lists)
    k = full.shape[1]
    mine_idx = lists[rank].to(full.device)
    mine = torch.zeros((per, k), dtype=full.dtype, device=full.device)
    mine[: len(mine_idx)] = full[mine_idx]
    if _rccl(dist) and full.device.type == "cuda":
        gathered = torch.empty((world * per, k), dtype=full.dtype, device=full.device)
        dist.all_gather_into_tensor(gathered, mine)
    else:
        gathered = _gather_host(dist, mine)
    for r in range(world):
        idx = lists[r].to(full.device)
        full[idx] = gathered[r * per: r * per + len(idx)]
    return full
