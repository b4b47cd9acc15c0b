"""Row-band sharding of ONE frame over ranks (the stretch goal).

RAFT-Stereo's correlation is a 1-D search along each image row, so the all-pairs volume, its pyramid and every
lookup are row-local: if rank r owns rows [a, b) of the frame, it can build its own slice of the correlation with
no communication at all.  Everything else in the network is a stencil over rows or a statistic over the image:

* a conv with kernel k / stride s / padding p / dilation d reads p rows above its band and up to d(k-1) - p rows
  below it -- those halo rows come from the neighbouring ranks (point-to-point send/recv, one message per
  neighbour and direction), rows outside the image are the conv's zero padding;
* ``avg_pool2d`` (pool2x), ``unfold`` (convex upsampling) are stencils the same way;
* a bilinear ``interpolate`` (align_corners) maps each fine row to a source row in GLOBAL coordinates, one row
  of halo on either side;
* instance norm (the feature encoder) needs the mean / variance over the whole image: the per-(n, c) sums and
  sums of squares are all-reduced (fp64) before the local rows are normalised.  Batch norm (eval) is local.

Rather than re-writing the network per band, :class:`RowBandMode` is a ``TorchFunctionMode`` that intercepts
exactly those functionals while the UNCHANGED oracle module (``models.raft_stereo.RAFTStereo``) runs on the
band: each intercepted call infers the tensor's pyramid level from its band height, exchanges the halo it needs
and runs the plain op on the extended rows.  Band boundaries are aligned to the coarsest GRU level
(2^(n_downsample + n_gru_layers - 1) rows at full resolution), so every stride-2 layer maps a band onto a band.
The result equals the single-process forward up to fp32 summation order (tests/test_rowband_cpu.py, gloo world
2 and 3), and the same code runs over RCCL on GPUs (P2P over xGMI).

480x640 fits one GPU trivially (the reference's fixed configuration, RAFTStereo/src/TRTRAFTStereo.cpp:13-14),
so this exists for frames too large for one device, not for the headline benchmark.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.overrides import TorchFunctionMode


@dataclass(frozen=True)
class RowBands:
    """Contiguous row bands of a height-``height`` frame over ``world`` ranks, boundaries at multiples of ``unit``
    (as even as the units allow; the first ranks get the extra units)."""
    height: int
    world: int
    unit: int

    def __post_init__(self):
        if self.height % self.unit:
            raise ValueError(f"height {self.height} is not a multiple of the band unit {self.unit}")
        if self.height // self.unit < self.world:
            raise ValueError(f"{self.height // self.unit} band units cannot feed {self.world} ranks")

    def band(self, rank: int) -> tuple[int, int]:
        units = self.height // self.unit
        q, r = divmod(units, self.world)
        start = rank * q + min(rank, r)
        n = q + (rank < r)
        return start * self.unit, (start + n) * self.unit


def raft_band_unit(cfg) -> int:
    """Full-resolution rows per band unit of a RAFT-Stereo config: the coarsest GRU level's stride."""
    return 2 ** (cfg.n_downsample + cfg.n_gru_layers - 1)


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


class RowBandMode(TorchFunctionMode):
    """Runs a module on this rank's row band [a, b) of a height-``height`` frame: halo-exchanging convs / pools /
    unfold / interpolate and globally normalised instance norm (see the module docstring)."""

    def __init__(self, bands: RowBands, rank: int, group=None, max_level: int = 8):
        super().__init__()
        self.bands, self.rank, self.world, self.group = bands, rank, bands.world, group
        self.a, self.b = bands.band(rank)
        # local band height -> (level, global start row, global height) at every power-of-two level
        self.levels = {}
        for lv in range(max_level + 1):
            f = 1 << lv
            if self.a % f or self.b % f or bands.height % f:
                break
            h = (self.b - self.a) // f
            if h < 1:
                break
            self.levels.setdefault(h, (lv, self.a // f, bands.height // f))
        self.messages = 0  # P2P messages sent (diagnostics)

    # -- geometry -------------------------------------------------------------------------------------------
    def _geom(self, x):
        h = x.shape[-2]
        if h not in self.levels:
            raise RuntimeError(f"tensor height {h} is not a band height of rank {self.rank} ({sorted(self.levels)})")
        return self.levels[h]

    # -- communication --------------------------------------------------------------------------------------
    def _exchange(self, x, top: int, bot: int):
        """Rows [a - top, a) from the previous rank and [b, b + bot) from the next one (zeros at the image edges)."""
        n, c, h, w = x.shape
        if top > h or bot > h:
            raise RuntimeError(f"halo ({top}, {bot}) rows exceeds the {h}-row band of rank {self.rank}")
        above = x.new_zeros(n, c, top, w)
        below = x.new_zeros(n, c, bot, w)
        ops = []
        r, world = self.rank, self.world
        if top > 0:
            if r + 1 < world:
                ops.append(dist.P2POp(dist.isend, x[:, :, h - top:].contiguous(), r + 1, self.group))
            if r > 0:
                ops.append(dist.P2POp(dist.irecv, above, r - 1, self.group))
        if bot > 0:
            if r > 0:
                ops.append(dist.P2POp(dist.isend, x[:, :, :bot].contiguous(), r - 1, self.group))
            if r + 1 < world:
                ops.append(dist.P2POp(dist.irecv, below, r + 1, self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
            self.messages += sum(1 for o in ops if o.op is dist.isend)
        return above, below

    def _extend(self, x, lo: int, hi: int):
        """Band-local rows covering GLOBAL rows [lo, hi) of x's level (halo exchanged, zero outside the image)."""
        _, start, _ = self._geom(x)
        h = x.shape[-2]
        top, bot = start - lo, hi - (start + h)
        above, below = self._exchange(x, max(top, 0), max(bot, 0))
        parts = []
        if top > 0:
            parts.append(above)
        core = x[:, :, max(-top, 0): h + min(bot, 0)]
        parts.append(core)
        if bot > 0:
            parts.append(below)
        return torch.cat(parts, dim=2) if len(parts) > 1 else core

    def _stencil_rows(self, x, k, s, p, d):
        """Extended input rows and the output band rows [o0, o1) of a k / s / p / d stencil over x's band."""
        lv, start, H = self._geom(x)
        h = x.shape[-2]
        if start % s or h % s:
            raise RuntimeError(f"stride {s} does not map rank {self.rank}'s band onto a band")
        o0, o1 = start // s, (start + h) // s
        lo, hi = o0 * s - p, (o1 - 1) * s - p + d * (k - 1) + 1
        return self._extend(x, lo, hi), o1 - o0

    # -- intercepted functionals ----------------------------------------------------------------------------
    def _conv2d(self, x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
        (sh, sw), (ph, pw), (dh, dw) = _pair(stride), _pair(padding), _pair(dilation)
        kh = weight.shape[-2]
        if kh == 1 and sh == 1 and ph == 0:
            return F.conv2d(x, weight, bias, (sh, sw), (ph, pw), (dh, dw), groups)
        xe, rows = self._stencil_rows(x, kh, sh, ph, dh)
        y = F.conv2d(xe, weight, bias, (sh, sw), (0, pw), (dh, dw), groups)
        assert y.shape[-2] == rows, (y.shape, rows)
        return y

    def _avg_pool2d(self, x, kernel_size, stride=None, padding=0, ceil_mode=False, count_include_pad=True,
                    divisor_override=None):
        (kh, kw) = _pair(kernel_size)
        (sh, sw) = _pair(stride if stride is not None else kernel_size)
        (ph, pw) = _pair(padding)
        if kh == 1 and sh == 1 and ph == 0:  # row-local (the correlation pyramid's [1, 2] pooling)
            return F.avg_pool2d(x, kernel_size, stride, padding, ceil_mode, count_include_pad, divisor_override)
        if ceil_mode or (ph > 0 and not count_include_pad):
            raise NotImplementedError("row-band avg_pool2d: floor mode with zero padding counted only")
        xe, rows = self._stencil_rows(x, kh, sh, ph, 1)
        y = F.avg_pool2d(xe, (kh, kw), (sh, sw), (0, pw), False, True, divisor_override)
        assert y.shape[-2] == rows
        return y

    def _unfold(self, x, kernel_size, dilation=1, padding=0, stride=1):
        (kh, kw), (dh, dw), (ph, pw), (sh, sw) = _pair(kernel_size), _pair(dilation), _pair(padding), _pair(stride)
        xe, rows = self._stencil_rows(x, kh, sh, ph, dh)
        return F.unfold(xe, (kh, kw), (dh, dw), (0, pw), (sh, sw))

    def _instance_norm(self, x, running_mean=None, running_var=None, weight=None, bias=None, use_input_stats=True,
                       momentum=0.1, eps=1e-5):
        if not use_input_stats:
            return F.instance_norm(x, running_mean, running_var, weight, bias, False, momentum, eps)
        _, _, H = self._geom(x)
        xd = x.double()
        s = torch.stack([xd.sum((2, 3)), (xd * xd).sum((2, 3))])  # [2, N, C]
        dist.all_reduce(s, group=self.group)
        cnt = float(H * x.shape[-1])
        mean = s[0] / cnt
        var = (s[1] / cnt - mean * mean).clamp_min(0.0)
        rstd = torch.rsqrt(var + eps)
        y = (x - mean.to(x.dtype)[..., None, None]) * rstd.to(x.dtype)[..., None, None]
        if weight is not None:
            y = y * weight[None, :, None, None]
        if bias is not None:
            y = y + bias[None, :, None, None]
        return y

    def _interpolate(self, x, size=None, scale_factor=None, mode="nearest", align_corners=None, **kw):
        if mode != "bilinear" or not align_corners or size is None:
            raise NotImplementedError("row-band interpolate: bilinear with align_corners and an explicit size")
        _, cs, Hc = self._geom(x)
        hf, wf = size
        if hf not in self.levels:
            raise RuntimeError(f"interpolate target height {hf} is not a band height of rank {self.rank}")
        _, fs, Hf = self.levels[hf]
        lc, lf = self.levels[x.shape[-2]][0], self.levels[hf][0]
        scale = torch.tensor((Hc - 1) / (Hf - 1) if Hf > 1 else 0.0, dtype=torch.float32)

        def src_rows(f0, f1):  # PyTorch's align_corners source rows (fp32, like its CPU kernel) of fine rows [f0, f1)
            src = torch.arange(f0, f1, dtype=torch.float32) * scale
            y0 = src.floor().long().clamp(max=Hc - 1)
            return src, y0, (y0 + 1).clamp(max=Hc - 1)

        # every rank exchanges the SAME halo (the largest any band needs), so the sends and receives pair up
        top = bot = 0
        for q in range(self.world):
            qa, qb = self.bands.band(q)
            _, q0, q1 = src_rows(qa >> lf, qb >> lf)
            top = max(top, (qa >> lc) - int(q0.min()))
            bot = max(bot, int(q1.max()) + 1 - (qb >> lc))
        src, y0, y1 = src_rows(fs, fs + hf)
        lo = cs - top
        xe = self._extend(x, lo, cs + x.shape[-2] + bot)
        lam = (src - y0.float()).to(device=x.device, dtype=x.dtype)
        r0, r1 = xe[:, :, (y0 - lo).to(x.device)], xe[:, :, (y1 - lo).to(x.device)]
        rows = r0 + (r1 - r0) * lam[None, None, :, None]
        return F.interpolate(rows, size=(hf, wf), mode="bilinear", align_corners=True)

    def __torch_function__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func is F.conv2d:
            return self._conv2d(*args, **kwargs)
        if func is F.avg_pool2d:
            return self._avg_pool2d(*args, **kwargs)
        if func is F.unfold:
            return self._unfold(*args, **kwargs)
        if func is F.instance_norm:
            return self._instance_norm(*args, **kwargs)
        if func is F.interpolate:
            return self._interpolate(*args, **kwargs)
        if func in (F.conv1d, F.conv3d, F.max_pool2d, F.adaptive_avg_pool2d, F.pad, F.group_norm, F.layer_norm):
            raise NotImplementedError(f"row-band sharding has no halo rule for {func.__name__}")
        return func(*args, **kwargs)


def raft_rowband_forward(model, image1, image2, iters=None, group=None, rank=None, world=None):
    """RAFT-Stereo forward of ONE frame sharded by rows over the process group.

    ``image1`` / ``image2``: the FULL frames [B, 3, H, W] (RGB 0..255; every rank passes the same frames and
    slices its own band; a caller that only holds its band rows uses :func:`raft_rowband_band`).  Returns this
    rank's band of ``flow_up`` [B, 1, b - a, W] and the band (a, b)."""
    rank = dist.get_rank(group) if rank is None else rank
    world = dist.get_world_size(group) if world is None else world
    bands = RowBands(image1.shape[2], world, raft_band_unit(model.cfg))
    a, b = bands.band(rank)
    return raft_rowband_band(model, image1[:, :, a:b], image2[:, :, a:b], bands, rank, iters, group), (a, b)


def raft_rowband_band(model, band1, band2, bands: RowBands, rank: int, iters=None, group=None):
    """The sharded forward on inputs that already are this rank's band rows."""
    with torch.no_grad(), RowBandMode(bands, rank, group):
        _, flow_up = model(band1, band2, iters=iters)
    return flow_up


def gather_bands(band_out, bands: RowBands, group=None):
    """All-gather the ranks' row bands of a [B, C, rows, W] output into the full [B, C, H, W] frame."""
    world = bands.world
    hmax = max(bands.band(r)[1] - bands.band(r)[0] for r in range(world))
    n, c, h, w = band_out.shape
    pad = band_out.new_zeros(n, c, hmax, w)
    pad[:, :, :h] = band_out
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:, :, : bands.band(r)[1] - bands.band(r)[0]] for r, p in enumerate(parts)], dim=2)


__all__ = ["RowBands", "RowBandMode", "raft_band_unit", "raft_rowband_forward", "raft_rowband_band", "gather_bands"]
