"""Frame sharding across GPUs — the replacement of Camera#render_fork +
fork_jobs (src/camera.rb:41-68, src/fork_jobs.rb:1-33).

The reference forks N processes, gives child i the contiguous column band
[floor(i/N*W), floor((i+1)/N*W)) and merges the children's JSON files.  Here
the frame is cut into ``tile_rows``-row tiles dealt round-robin (tile t ->
rank t % N, which balances glass/mirror-heavy regions that contiguous bands
pile onto one child), each rank renders its tiles into a packed device buffer
(``rtx_render_tiles_device``), and ONE gather over RCCL/xGMI brings the packed
buffers to rank 0, which scatters the rows into the frame.  Pixels are
independent and every pixel's result is keyed only by (seed, x, y, sample,
path), so the frame is bit-identical for every N.
"""

import numpy as np

DEFAULT_TILE_ROWS = 8


def rows_per_rank(height, tile_rows, nranks):
    tiles = (height + tile_rows - 1) // tile_rows
    return ((tiles + nranks - 1) // nranks) * tile_rows


def rank_rows(height, tile_rows, rank, nranks):
    """Image row y of every packed row of `rank` (-1 = padding past the bottom)."""
    n = rows_per_rank(height, tile_rows, nranks)
    k = np.arange(n) // tile_rows
    y = (k * nranks + rank) * tile_rows + np.arange(n) % tile_rows
    y[y >= height] = -1
    return y


def unpack_index(height, tile_rows, nranks):
    """For the rank-major concatenation of all packed buffers: (source row, image row) pairs."""
    src, dst = [], []
    n = rows_per_rank(height, tile_rows, nranks)
    for r in range(nranks):
        y = rank_rows(height, tile_rows, r, nranks)
        keep = y >= 0
        src.append(np.nonzero(keep)[0] + r * n)
        dst.append(y[keep])
    return np.concatenate(src), np.concatenate(dst)


def row_tile_costs(tile_rays, tile_rows):
    """Per tile_rows-row tile: the rays of its 8x8 tiles (Renderer.tile_rays(),
    [ceil(H/8), ceil(W/8)]); tile_rows must be a multiple of 8."""
    if tile_rows % 8:
        raise ValueError("cost-balanced tiles need tile_rows a multiple of 8")
    m = tile_rows // 8
    per_band = np.asarray(tile_rays, np.int64).sum(axis=1)
    n = (len(per_band) + m - 1) // m
    return np.array([per_band[k * m:(k + 1) * m].sum() for k in range(n)], np.int64)


def lpt_plan(costs, nranks):
    """Longest-processing-time split of tiles over ranks: tiles by decreasing
    cost (ties: lower index first), each to the rank with the least total so
    far (ties: lower rank).  Deterministic, so every rank computes the same
    plan from the same costs.  Returns nranks lists of tile indices (each
    ascending), padded to one length with len(costs) (past the bottom)."""
    costs = np.asarray(costs, np.int64)
    n = len(costs)
    order = sorted(range(n), key=lambda t: (-int(costs[t]), t))
    load = [0] * nranks
    lists = [[] for _ in range(nranks)]
    for t in order:
        r = min(range(nranks), key=lambda k: (load[k], len(lists[k]), k))
        lists[r].append(t)
        load[r] += int(costs[t])
    width = max(len(l) for l in lists)
    return [sorted(l) + [n] * (width - len(l)) for l in lists]


def plan_unpack_index(plan, height, tile_rows):
    """(source row, image row) pairs of the rank-major concatenation of the packed
    buffers of a tile-list plan (rows_per_rank = len(plan[0]) * tile_rows)."""
    n = len(plan[0]) * tile_rows
    src, dst = [], []
    for r, tiles in enumerate(plan):
        for k, t in enumerate(tiles):
            for j in range(tile_rows):
                y = t * tile_rows + j
                if y < height:
                    src.append(r * n + k * tile_rows + j)
                    dst.append(y)
    return np.array(src, np.int64), np.array(dst, np.int64)


def unpack(gathered, height, tile_rows, nranks):
    """gathered: [nranks * rows_per_rank, W, 3] (numpy or torch) -> frame [H, W, 3]."""
    src, dst = unpack_index(height, tile_rows, nranks)
    try:
        import torch
        if isinstance(gathered, torch.Tensor):
            out = torch.empty((height,) + tuple(gathered.shape[1:]), dtype=gathered.dtype, device=gathered.device)
            s = torch.as_tensor(src, device=gathered.device)
            d = torch.as_tensor(dst, device=gathered.device)
            out.index_copy_(0, d, gathered.index_select(0, s))
            return out
    except ImportError:
        pass
    out = np.empty((height,) + tuple(gathered.shape[1:]), dtype=gathered.dtype)
    out[dst] = gathered[src]
    return out


class DistributedFrame:
    """One rank's share of tile-sharded rendering + the RCCL gather to rank 0.

    Needs an initialized torch.distributed process group (``nccl`` = RCCL on
    ROCm, or ``gloo`` for CPU tests).  The caller renders this rank's tiles
    into ``packed`` ([rows_per_rank, W, 3] float64), then either ``gather()``
    (blocking) or, to overlap frame i's gather with frame i + 1's render,
    ``h = gather_start()`` ... render the next frame into the new ``packed``
    ... ``gather_finish(h)``.  With ``buffers=2`` the packed buffers alternate,
    so the render of frame i + 1 never writes the buffer frame i's gather
    reads; rank 0's unpack of frame i is queued on the caller's stream before
    the gather of frame i + 1 is issued (a collective waits for the stream it
    is issued from), so the single receive buffer is never overwritten early."""

    def __init__(self, width, height, tile_rows, rank, nranks, device, buffers=1, force_collective=False, plan=None):
        import torch
        self.width, self.height = width, height
        self.tile_rows, self.rank, self.nranks = tile_rows, rank, nranks
        # plan: per-rank tile lists (lpt_plan) instead of round-robin tiles
        self.plan = plan
        # force_collective: issue the gather even with one rank (the GPU test of
        # the multi-rank path runs it under a 1-rank RCCL group)
        self.collective = nranks > 1 or force_collective
        self.rows = len(plan[0]) * tile_rows if plan else rows_per_rank(height, tile_rows, nranks)
        self.bufs = [torch.zeros((self.rows, width, 3), dtype=torch.float64, device=device)
                     for _ in range(max(1, buffers))]
        self._i = 0
        self.packed = self.bufs[0]
        self.gathered = None
        if rank == 0:
            self.gathered = torch.zeros((nranks * self.rows, width, 3), dtype=torch.float64, device=device)
            src, dst = plan_unpack_index(plan, height, tile_rows) if plan else unpack_index(height, tile_rows, nranks)
            self.src = torch.as_tensor(src, device=device)
            self.dst = torch.as_tensor(dst, device=device)
            self.frame = torch.zeros((height, width, 3), dtype=torch.float64, device=device)

    def gather_start(self, buf=None):
        """Start ONE collective (every rank's packed tiles to rank 0) without
        waiting for it.  Without ``buf``: gather ``packed`` and move ``packed``
        to the next buffer; with ``buf``: gather that one (the caller manages
        the buffers and their reuse)."""
        import torch.distributed as dist
        advance = buf is None
        buf = self.packed if buf is None else buf
        work = None
        if self.collective:
            chunks = list(self.gathered.chunk(self.nranks, 0)) if self.rank == 0 else None
            work = dist.gather(buf, chunks, dst=0, async_op=True)
        if advance:
            self._i = (self._i + 1) % len(self.bufs)
            self.packed = self.bufs[self._i]
        return work, buf

    def gather_finish(self, handle):
        """Wait for a started gather (the caller's stream waits for it); rank 0
        unpacks the rows and returns the frame."""
        work, buf = handle
        if work is not None:
            work.wait()
        if self.rank == 0:
            src = self.gathered if self.collective else buf
            self.frame.index_copy_(0, self.dst, src.index_select(0, self.src))
            return self.frame
        return None

    def gather(self):
        """ONE collective: every rank's packed tiles to rank 0; rank 0 returns the frame."""
        return self.gather_finish(self.gather_start())


class PipelinedTiles:
    """The multi-GPU frame step of bench.py (C3), frames pipelined: F renderers
    (contexts) on F streams, frame i on context j = i mod F renders this rank's
    tiles into packed buffer j; the current stream waits for it, finishes frame
    i - 1's gather (rank 0 unpacks it; buffer j' may be rendered into again
    after that, ``free_ev``), then starts frame i's gather asynchronously, so it
    overlaps frame i + 1's render.  ``drain()`` finishes the last gather.

    renderers: raytracing_rb_amd.runtime.Renderer, one per frame in flight;
    streams: torch.cuda.Stream per renderer; on_frame(i, frame): rank 0's
    callback with frame i (the DistributedFrame's frame tensor, reused)."""

    def __init__(self, renderers, streams, width, height, tile_rows, rank, nranks, device, seed=1,
                 force_collective=False, on_frame=None, plan=None):
        import torch
        self.rs, self.streams = renderers, streams
        self.F = len(renderers)
        assert len(streams) == self.F
        self.tile_rows, self.rank, self.nranks, self.seed = tile_rows, rank, nranks, seed
        self.plan = plan
        self.stream = torch.cuda.current_stream(device)
        self.df = DistributedFrame(width, height, tile_rows, rank, nranks, device, buffers=self.F,
                                   force_collective=force_collective, plan=plan)
        self.pending = []
        self.free_ev = [None] * self.F
        self.on_frame = on_frame
        self.i = 0              # frames started
        self.done = 0           # frames gathered

    def _finish_one(self):
        import torch
        h, jj = self.pending.pop(0)
        frame = self.df.gather_finish(h)
        if self.on_frame is not None and self.rank == 0:
            self.on_frame(self.done, frame)
        self.done += 1
        ev = torch.cuda.Event()
        ev.record(self.stream)
        self.free_ev[jj] = ev

    def step(self):
        import torch
        j = self.i % self.F
        self.i += 1
        # Buffer j may still be read by a started gather (always so with F = 1):
        # finish gathers until none reads it, so its free event exists and the
        # render below is ordered after the gather.
        while any(jj == j for _, jj in self.pending):
            self._finish_one()
        if self.free_ev[j] is not None:
            self.streams[j].wait_event(self.free_ev[j])
        self.render_share(j)
        done = torch.cuda.Event()
        done.record(self.streams[j])
        while self.pending:
            self._finish_one()
        self.stream.wait_event(done)
        self.pending.append((self.df.gather_start(self.df.bufs[j]), j))

    def render_share(self, j, buf=None):
        """This rank's share of one frame into packed buffer j (or `buf`) on stream j."""
        ptr = (self.df.bufs[j] if buf is None else buf).data_ptr()
        if self.plan:
            self.rs[j].render_tile_list_device(ptr, self.plan[self.rank], self.tile_rows, seed=self.seed,
                                               stream=self.streams[j].cuda_stream)
        else:
            self.rs[j].render_tiles_device(ptr, self.tile_rows, self.rank, self.nranks, seed=self.seed,
                                           stream=self.streams[j].cuda_stream)

    def drain(self):
        while self.pending:
            self._finish_one()
