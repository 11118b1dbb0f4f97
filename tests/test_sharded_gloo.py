"""world_size-2 gloo run of the multi-GPU choreography (depthmapx_amd/sharded.py) on CPU.

Each rank builds the makeGraph shard for its source range, the shards are all-gathered as ragged
byte blobs and reassembled, each rank runs VGA global for its sources, and the 7 columns are
all-gathered.  The per-rank compute here is the C restatement (no GPU in this container); the
collectives, sharding and reassembly are exactly the code bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from golden_io import case_input_lines, load_case


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pack(g, n):
    bins = np.ascontiguousarray(g["bins"], dtype=np.int32)
    runs = np.ascontiguousarray(g["runs"], dtype=np.int16)
    hdr = np.array([n, len(runs)], dtype=np.int64)
    return np.concatenate([hdr.view(np.uint8), bins.view(np.uint8).ravel(), runs.view(np.uint8).ravel()])


def _unpack(buf):
    n, nr = np.frombuffer(buf[:16].tobytes(), dtype=np.int64)
    bins = np.frombuffer(buf[16:16 + n * 32 * 16].tobytes(), dtype=np.int32).reshape(n, 32, 4)
    runs = np.frombuffer(buf[16 + n * 32 * 16:16 + n * 32 * 16 + nr * 8].tobytes(), dtype=np.int16).reshape(nr, 4)
    return bins, runs


class _HostShard:
    """The Graph shard's blob interface (blob_size / write_blob_device) over a host byte array."""

    def __init__(self, buf):
        self.buf = buf

    def blob_size(self):
        return len(self.buf)

    def write_blob_device(self, ptr, n):
        import ctypes
        assert n == len(self.buf)
        ctypes.memmove(ptr, self.buf.ctypes.data, n)


class _HostAssembler:
    """PointMap.assemble over host pointers: unpack each rank's blob, concatenate in rank order."""

    def assemble(self, ctx, ptrs, sizes):
        import ctypes
        parts = [_unpack(np.frombuffer(ctypes.string_at(p, n), dtype=np.uint8)) for p, n in zip(ptrs, sizes)]
        return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle")):
        sys.path.insert(0, p)
    from depthmapx_amd.sharded import allgather_rows_chunked, choose_mk_mode, exchange_graph, shard_range, vga_nodes
    from pyoracle import OracleMap
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    meta, _ = load_case("syn16")
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    om.fill(*meta["fills"][0])
    om.make_graph()                       # index nodes
    N = om.num_nodes
    b, e = shard_range(N, rank, world)
    om.make_graph(node_begin=b, node_end=e)
    full = om.graph()
    ro = int(full["bins"][:b, :, 3].sum())
    nr = int(full["bins"][b:e, :, 3].sum())
    shard = _HostShard(_pack(dict(bins=full["bins"][b:e], runs=full["runs"][ro:ro + nr]), e - b))
    (bins, runs), xt = exchange_graph(_HostAssembler(), None, shard, dist, torch.device("cpu"))
    assert xt["bytes"] >= shard.blob_size() and xt["allgather_s"] >= 0
    om.set_graph(bins, runs)
    # --mk-mode auto: ranks measure different times but must take the same branch
    mode, dec = choose_mk_mode(dist, torch.device("cpu"), world, 1.0 + rank, 0.5 * rank, (e - b) / N)
    # the sharded step's symmetry scatter (VGA preparation) counts against sharding: a large one flips it
    mode_sym, dec_sym = choose_mk_mode(dist, torch.device("cpu"), world, 1.0 + rank, 0.5 * rank, (e - b) / N,
                                       100.0 * (rank + 1))
    assert mode_sym == "replicate" and dec_sym["sym_shard_s"] == 100.0 * world
    out = torch.full((N, 7), -1.0)
    # VGA sources: 16-node chunks dealt round-robin (bench.py uses 4096)
    mine = vga_nodes(N, rank, world, chunk=16)
    for c0 in range(0, len(mine), 16):
        cb, ce = int(mine[c0]), int(mine[min(c0 + 16, len(mine)) - 1]) + 1
        out[cb:ce] = torch.from_numpy(om.vga_global(node_begin=cb, node_end=ce)[cb:ce])
    allgather_rows_chunked(out, N, dist, chunk=16)
    q.put((rank, bins, runs, out.numpy(), mode, dec))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_multi_rank_gloo_matches_single_process(world):
    """World 2 and 4 (the 4-rank one-GPU rehearsal's shard ranges, blob sizes and row lists, DESIGN.md
    section 5) through the same helpers bench.py runs."""
    from pyoracle import OracleMap
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    meta, A = load_case("syn16")
    om = OracleMap(meta["region"], meta["spacing"], case_input_lines(meta))
    om.fill(*meta["fills"][0])
    om.make_graph()
    g = om.graph()
    ref = om.vga_global()
    # every rank measured mk = 1 + rank, exchange = 0.5 rank: the decision uses the max over ranks
    assert len({r[4] for r in res}) == 1 and res[0][5]["mk_shard_s"] == float(world)
    assert res[0][5]["exchange_s"] == 0.5 * (world - 1)
    assert res[0][4] == "shard"       # world + 0.5 (world - 1) < world / (1 / world)
    for _, bins, runs, out, _, _ in res:
        np.testing.assert_array_equal(bins, g["bins"])
        np.testing.assert_array_equal(runs, g["runs"])
        np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))
        np.testing.assert_array_equal(out.view(np.uint32), A["vga"].view(np.uint32))


@pytest.mark.parametrize("n,world,chunk", [(0, 2, 4), (1, 2, 4), (7, 3, 2), (65025, 8, 4096), (998001, 8, 4096)])
def test_vga_node_chunks_partition(n, world, chunk):
    from depthmapx_amd.sharded import vga_nodes
    parts = [vga_nodes(n, r, world, chunk) for r in range(world)]
    allv = np.sort(np.concatenate(parts)) if n else np.zeros(0, dtype=np.int64)
    np.testing.assert_array_equal(allv, np.arange(n))
    if n >= world * chunk * 4:
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= chunk


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 3), (65025, 8)])
def test_shard_ranges_partition(n, world):
    from depthmapx_amd.sharded import shard_range
    r = [shard_range(n, i, world) for i in range(world)]
    assert r[0][0] == 0 and r[-1][1] == n
    assert all(r[i][1] == r[i + 1][0] for i in range(world - 1))
    assert max(e - b for b, e in r) - min(e - b for b, e in r) <= 1
