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
