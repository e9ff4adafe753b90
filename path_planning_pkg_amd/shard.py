"""Row-block sharding of the map build across ranks (BASELINE.json cfg4).

The reference builds Grid2D's log-odds map (`Grid2D.cpp:99-208`) on one core.  Here rank r of
G builds only rows [r0, r1) of a planner's map (hastar_set_row_window: decay and the box/line
rasters skip the other rows), exports its block into a device buffer, the blocks are
all-gathered over RCCL (xGMI), and every rank imports the whole map.  Each cell's update
sequence is the reference's, so the gathered map equals the single-GPU build bit for bit
(tests/test_gpu_parity.py::test_row_sharded_map_build).

`update_goal` (relocate, `Grid3D.cpp:169-203`) is a global rotation and stays unsharded: it
runs on every rank before the window is set.
"""
import torch


def row_blocks(N, world):
    """Equal-height contiguous row blocks (the last may be short or empty):
    [(r0, r1)] per rank, and R = rows per block (all-gather needs equal chunks)."""
    if N < 0 or world < 1:
        raise ValueError("need N >= 0 and world >= 1")
    R = -(-N // world)
    return [(min(r * R, N), min((r + 1) * R, N)) for r in range(world)], R


def gather_rows(local, world, group=None):
    """All-gather equal-size row blocks (world = 1: the block itself)."""
    if world == 1:
        return local
    import torch.distributed as dist
    out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, local, group=group)
    return out


def drive_sharded(planner, proto, rank, world, device, group=None, reset=True):
    """tests/scenarios.py::drive with the map build row-sharded over `world` ranks.
    Every rank calls this for the same planner inputs; afterwards every rank's planner holds
    the full map.  Returns the gathered map as a flat device tensor (N*N floats)."""
    N = planner.N
    blocks, R = row_blocks(N, world)
    r0, r1 = blocks[rank]
    planner.update_goal(proto["goal"], proto["start"])
    planner.set_row_window(r0, r1)
    try:
        for _ in range(proto["cycles"]):
            planner.decay()
            if len(proto["lines"]):
                planner.update_lines(proto["lines"], [proto["line_conf"]] * len(proto["lines"]), proto["line_width"])
            if len(proto["boxes"]):
                planner.update_boxes(proto["boxes"], [proto["box_conf"]] * len(proto["boxes"]), proto["apf_r"])
    finally:
        planner.set_row_window(0, N)
    local = torch.zeros(R * N, dtype=torch.float32, device=device)
    if local.is_cuda:
        torch.cuda.synchronize(device)  # the zero fill runs on torch's stream
    planner.export_rows(r0, r1, local.data_ptr())
    full = gather_rows(local, world, group)
    if full.is_cuda:
        torch.cuda.synchronize(device)
    planner.import_rows(0, N, full.data_ptr())
    if reset:
        planner.reset()
    return full[: N * N]


# ---- the backward grid-distance field, row-sharded (include/hastar.h: hastar_field_rows) ----
# BASELINE.json's north_star: "the Grid2D obstacle inflation + backward-Dijkstra heuristic
# precompute shards across GPUs with an RCCL all-gather over xGMI".  Rank r relaxes rows
# [r0, r1) of the field (csrc/hastar_field.hip) against two halo rows, the ranks all-gather their
# blocks' first and last rows, and every rank whose halo changed relaxes again, until no block
# edge changes.  The field's equations have one solution, so the result equals the one-GPU field
# bit for bit whatever the split (tests/test_gpu_field.py, tests/test_multirank.py).

def _planner_relax(planner):
    def relax(buf, r0, r1, init, halo_changed):
        if buf.is_cuda:
            torch.cuda.synchronize(buf.device)  # buffer writes on torch's stream come first
        return planner.field_rows(buf.data_ptr(), r0, r1, init, halo_changed)
    return relax


def _halo_updates(edges, rank, blocks, N):
    """From the all-gathered [first row, last row, changed mask] of every rank: this rank's new
    upper / lower halo rows (or None when unchanged) and its halo_changed bits."""
    up = dn = None
    bits = 0
    r0, r1 = blocks[rank]
    if rank > 0 and blocks[rank - 1][1] > blocks[rank - 1][0] and int(edges[rank - 1, 2 * N]) & 4:
        up, bits = edges[rank - 1, N:2 * N], bits | 1
    if rank + 1 < len(blocks) and blocks[rank + 1][1] > blocks[rank + 1][0] and int(edges[rank + 1, 2 * N]) & 2:
        dn, bits = edges[rank + 1, :N], bits | 2
    return up, dn, bits


def heuristic_field_sharded(planner, rank, world, device, group=None, relax=None, max_rounds=1 << 20):
    """Every rank calls this for the same planner state (the whole map and goal on every rank:
    drive_sharded leaves them there).  Returns (full field as a flat device tensor of N*N floats,
    exchange rounds, relaxation passes of this rank)."""
    import torch.distributed as dist
    N = planner.N
    blocks, R = row_blocks(N, world)
    r0, r1 = blocks[rank]
    relax = relax or _planner_relax(planner)
    buf = torch.empty((R + 2) * N, dtype=torch.float32, device=device)
    mine = r1 > r0
    init, bits, rounds, passes = True, 0, 0, 0
    while True:
        mask = 0
        if mine:
            mask, p = relax(buf, r0, r1, init, bits)
            passes += p
        init = False
        rounds += 1
        if world == 1:
            break  # no neighbours: the block's first relaxation is the field
        local = torch.empty(2 * N + 1, dtype=torch.float32, device=device)
        if mine:
            local[:N] = buf[N:2 * N]
            local[N:2 * N] = buf[(r1 - r0) * N:(r1 - r0 + 1) * N]
        else:
            local[:2 * N] = float("inf")
        local[2 * N] = float(mask)
        edges = torch.empty(world * (2 * N + 1), dtype=torch.float32, device=device)
        if world > 1:
            dist.all_gather_into_tensor(edges, local, group=group)
        else:
            edges.copy_(local)
        edges = edges.view(world, 2 * N + 1)
        if not any(int(m) & 6 for m in edges[:, 2 * N].tolist()) or rounds >= max_rounds:
            break  # no block edge changed: every halo is final
        up, dn, bits = _halo_updates(edges, rank, blocks, N)
        if up is not None:
            buf[:N] = up
        if dn is not None:
            buf[(r1 - r0 + 1) * N:(r1 - r0 + 2) * N] = dn
    block = torch.full((R * N,), float("inf"), dtype=torch.float32, device=device)
    if mine:
        block[:(r1 - r0) * N] = buf[N:(r1 - r0 + 1) * N]
    full = gather_rows(block, world, group)
    if full.is_cuda:
        torch.cuda.synchronize(device)
    return full[: N * N], rounds, passes


def heuristic_field_standins(planner, world, device):
    """The same protocol with `world` stand-in ranks in one process on one device (a one-GPU box
    rehearses the sharded precompute): per round every block relaxes, then the edge rows move.
    Returns (full field, rounds, passes summed over the stand-ins)."""
    N = planner.N
    blocks, R = row_blocks(N, world)
    relax = _planner_relax(planner)
    bufs = [torch.empty((R + 2) * N, dtype=torch.float32, device=device) for _ in range(world)]
    bits = [0] * world
    init, rounds, passes = True, 0, 0
    while True:
        edges = torch.empty((world, 2 * N + 1), dtype=torch.float32, device=device)
        for r, (r0, r1) in enumerate(blocks):
            mask = 0
            if r1 > r0:
                mask, p = relax(bufs[r], r0, r1, init, bits[r])
                passes += p
                edges[r, :N] = bufs[r][N:2 * N]
                edges[r, N:2 * N] = bufs[r][(r1 - r0) * N:(r1 - r0 + 1) * N]
            else:
                edges[r, :2 * N] = float("inf")
            edges[r, 2 * N] = float(mask)
        init = False
        rounds += 1
        if not any(int(m) & 6 for m in edges[:, 2 * N].tolist()):
            break
        for r, (r0, r1) in enumerate(blocks):
            if r1 <= r0:
                continue
            up, dn, bits[r] = _halo_updates(edges, r, blocks, N)
            if up is not None:
                bufs[r][:N] = up
            if dn is not None:
                bufs[r][(r1 - r0 + 1) * N:(r1 - r0 + 2) * N] = dn
    full = torch.full((N * N,), float("inf"), dtype=torch.float32, device=device)
    for r, (r0, r1) in enumerate(blocks):
        if r1 > r0:
            full[r0 * N:r1 * N] = bufs[r][N:(r1 - r0 + 1) * N]
    if full.is_cuda:
        torch.cuda.synchronize(device)
    return full, rounds, passes
