"""Multi-GPU frame assembly: pixel-row shards -> one RCCL all-gather -> full frame.

The reference renders one frame in one process with OpenMP over pixels
(src/core/scene.cpp:31).  Here each rank (one MI355X, one process) renders the rows
whose (row / row_block) % world == rank (include/rt_hw.h rt_params); rows are interleaved
in blocks so every rank gets a similar mix of cheap and expensive image regions.  Pixel
results do not depend on the partition (per-pixel RNG), so the gathered frame is
bitwise identical for any world size.

The only collective is one all_gather of each rank's float sums (24.9 MB at 1080p),
padded to the largest shard; RCCL over xGMI when the tensors live on the GPU ("nccl"
backend), gloo on CPU tensors in the tests.
"""
import torch
import torch.distributed as dist


def shard_row_ids(height, rank, world, row_block=8):
    return [r for r in range(height) if (r // row_block) % world == rank]


def max_shard_rows(height, world, row_block=8):
    return max(len(shard_row_ids(height, r, world, row_block)) for r in range(world))


def gather_frame(local, height, width, rank, world, row_block=8, out=None, group=None):
    """local: (max_rows * width * 3,) tensor holding this rank's rows (padded): the float
    sums, or the 8-bit finished rows (rt_tonemap_u8_device, 4x fewer bytes on the wire).
    Returns the (height, width, 3) frame (on every rank) in row order."""
    max_rows = max_shard_rows(height, world, row_block)
    assert local.numel() == max_rows * width * 3, (local.numel(), max_rows, width)
    if world == 1:
        frame = local.view(max_rows, width, 3)[:height]
        return frame if out is None else out.copy_(frame)
    buf = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    if hasattr(dist, "all_gather_into_tensor") and local.device.type == "cuda":
        dist.all_gather_into_tensor(buf, local, group=group)
    else:
        dist.all_gather(list(buf.chunk(world)), local, group=group)
    parts = buf.view(world, max_rows, width, 3)
    frame = out if out is not None else torch.empty((height, width, 3), dtype=local.dtype, device=local.device)
    for r in range(world):
        rows = shard_row_ids(height, r, world, row_block)
        idx = torch.tensor(rows, dtype=torch.long, device=local.device)
        frame.index_copy_(0, idx, parts[r, :len(rows)])
    return frame
