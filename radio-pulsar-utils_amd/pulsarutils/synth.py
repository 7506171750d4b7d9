"""Deterministic synthetic filterbanks for the C1-C5 parity / benchmark configs.

SURVEY.md §8d fixes the recipe of each config.  Two generators exist:

* :func:`rfi_filterbank_np` - numpy, host side, bit-reproducible from a seed
  (``np.random.default_rng``).  Used for the C4 cleaning goldens and the CPU
  parity subsets.
* :func:`pulsar_filterbank_device` - torch, generated channel block by channel
  block directly in HBM (C2/C3/C5 are 4-17 GB; they never touch host memory).

Every generator injects a unit dispersed pulse at ``nsamples // 2`` using the
reference's own delay convention (``simulate.py:20-22``: channel ``i`` is rolled by
``+shift_i``), so the dedispersed series peaks at the pulse DM.
"""
import numpy as np

from .configs import Config


def _shifts(cfg: Config, dm: float) -> np.ndarray:
    from .dedispersion import dedispersion_shifts
    return dedispersion_shifts(cfg.nchan, dm, cfg.start_freq, cfg.bandwidth, cfg.tsamp).astype(np.int64)


def rfi_filterbank_np(cfg: Config, dtype: str = None, seed: int = None) -> np.ndarray:
    """C4-style RFI-heavy filterbank, float32 or uint8.

    Base: per-channel bandpass level 64*b_c with noise sigma 8*b_c.  RFI: 5 % of
    channels at 3x the mean, 3 % at 4x the variance, 20 broadband zero-DM spikes
    (+10 sigma over 1-16 samples), one narrow-band periodic tone, plus a dispersed
    pulse (+2 sigma) at ``cfg.pulse_dm``.  uint8 = ``clip(rint(x), 0, 255)``.
    """
    dtype = dtype or cfg.dtype
    rng = np.random.default_rng(cfg.seed if seed is None else seed)
    nchan, n = cfg.nchan, cfg.nsamples
    chans = np.arange(nchan)
    band = (1.0 + 0.3 * np.sin(np.pi * chans / nchan)).astype(np.float32)
    level = 64.0 * band
    sigma = 8.0 * band
    hot = rng.choice(nchan, max(1, nchan * 5 // 100), replace=False)
    level[hot] *= 3.0
    noisy = rng.choice(nchan, max(1, nchan * 3 // 100), replace=False)
    sigma[noisy] *= 2.0
    x = rng.standard_normal((nchan, n), dtype=np.float32)
    x *= sigma[:, None]
    x += level[:, None]
    # broadband zero-DM spikes
    for _ in range(20):
        t0 = int(rng.integers(0, n - 16))
        w = int(rng.integers(1, 17))
        x[:, t0:t0 + w] += 10.0 * sigma[:, None]
    # narrow-band periodic tone
    tone_chan = int(rng.integers(0, nchan))
    t = np.arange(n, dtype=np.float32)
    x[tone_chan] += 3.0 * sigma[tone_chan] * np.sin(2 * np.pi * t / 37.0).astype(np.float32)
    # dispersed pulse
    sh = _shifts(cfg, cfg.pulse_dm)
    x[chans, (n // 2 + sh) % n] += 2.0 * sigma
    if dtype == "u8":
        np.rint(x, out=x)
        np.clip(x, 0, 255, out=x)
        return x.astype(np.uint8)
    if dtype == "f64":
        return x.astype(np.float64)
    return x


def pulsar_filterbank_device(cfg: Config, device="cuda", dtype: str = None, block: int = 64,
                             seed: int = None):
    """Noise + unit dispersed pulse, generated in HBM.

    float32: ``|N(0, 0.5)|`` + 1.0 at the dispersed pulse position.
    uint8:   ``clip(rint(64 + 8 N(0,1)), 0, 255)`` + 16 at the pulse.
    Returns a contiguous ``(nchan, nsamples)`` torch tensor on ``device``.
    """
    import torch
    dtype = dtype or cfg.dtype
    g = torch.Generator(device=device)
    g.manual_seed(cfg.seed if seed is None else seed)
    nchan, n = cfg.nchan, cfg.nsamples
    tdt = {"f32": torch.float32, "u8": torch.uint8, "f64": torch.float64}[dtype]
    out = torch.empty((nchan, n), dtype=tdt, device=device)
    sh = torch.as_tensor(_shifts(cfg, cfg.pulse_dm), device=device)
    pos = (n // 2 + sh) % n
    for c0 in range(0, nchan, block):
        c1 = min(nchan, c0 + block)
        z = torch.randn((c1 - c0, n), generator=g, device=device, dtype=torch.float32)
        rows = torch.arange(c1 - c0, device=device)
        if dtype == "u8":
            z.mul_(8.0).add_(64.0)
            z[rows, pos[c0:c1]] += 16.0
            out[c0:c1] = z.round_().clamp_(0, 255).to(torch.uint8)
        else:
            z.abs_().mul_(0.5)
            z[rows, pos[c0:c1]] += 1.0
            out[c0:c1] = z.to(tdt)
    return out
