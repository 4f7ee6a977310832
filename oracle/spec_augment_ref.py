"""CPU restatement of SpecAugment -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (liteasr_amd/utils/transform/spec_augment.py + the HIP kernels in
liteasr_amd/csrc/specaug.hip) never does.

Follows liteasr/utils/transform/spec_augment.py:14-125 (reference) in two halves:

* ``draw_plan`` consumes the process-global ``random`` and ``numpy.random`` streams in
  exactly the reference's order (time_warp :30-32, freq_mask :60-65, time_mask :93-101)
  and records the integers it drew as a plan: (center, warped) and the clipped
  [lo, hi) mask ranges.
* ``apply_plan`` applies a plan to one (time, freq) float32 utterance.

The time warp resizes the two segments with Pillow's BICUBIC filter.  Pillow is a
third-party dependency of the reference (not vendored under /root/reference; Pillow 12.2.0
in this image).  Its published float32 ('F' mode) algorithm is restated here: separable
resampling (libImaging/Resample.c, ``precompute_coeffs`` + ``ImagingResampleVertical_32bpc``):
for output row yy of an (in -> out) resize, scale = in/out, filterscale = max(scale, 1),
support = 2*filterscale, center = (yy+0.5)*scale, taps y in [int(center-support+0.5),
int(center+support+0.5)) clipped to [0, in), weight w(y) = bicubic((y-center+0.5)/
filterscale) with a = -0.5, normalised by their sum; the output is the double-precision
sum of pixel*weight in tap order, rounded to float32.  Only the vertical pass runs (the
width is unchanged) and an equal-size resize is a copy (Image.resize).  This restatement
is pinned bit-exactly against Pillow itself by tests/test_oracle_golden.py, and the whole
transform against the reference's SpecAugment by tests/golden/spec_aug.npz.

The mean fill follows numpy's ``ndarray.mean`` of a float32 array (float32 pairwise sum);
the restatement sums in float64 instead, so filled values agree to ~1e-7 relative.
"""

import random

import numpy as np


def bicubic(x):
    # Resample.c bicubic_filter, a = -0.5
    a = -0.5
    if x < 0.0:
        x = -x
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def resize_rows(src, out_rows):
    """Pillow BICUBIC resize of an (in_rows, F) float32 'F' image to (out_rows, F)."""
    src = np.ascontiguousarray(src, dtype=np.float32)
    n_in = src.shape[0]
    if n_in == out_rows:
        return src.copy()
    scale = float(n_in) / out_rows
    fscale = max(scale, 1.0)
    support = 2.0 * fscale
    out = np.empty((out_rows, src.shape[1]), np.float32)
    s64 = src.astype(np.float64)
    for yy in range(out_rows):
        center = (yy + 0.5) * scale
        ss = 1.0 / fscale
        lo = max(int(center - support + 0.5), 0)
        hi = min(int(center + support + 0.5), n_in)
        w = [bicubic((y - center + 0.5) * ss) for y in range(lo, hi)]
        ww = 0.0
        for v in w:
            ww += v
        if ww != 0.0:
            w = [v / ww for v in w]
        acc = np.zeros(src.shape[1], np.float64)
        for i, y in enumerate(range(lo, hi)):
            acc = acc + s64[y] * w[i]
        out[yy] = acc.astype(np.float32)
    return out


def draw_plan(t, f, cfg):
    """Draw one utterance's random numbers exactly as SpecAugment.__call__ does."""
    warp = None
    window = cfg.time_warp
    if not (t - window <= window):
        center = random.randrange(window, t - window)
        warped = random.randrange(center - window, center + window) + 1
        warp = (center, warped)
    fmasks = []
    for fw, raw in np.random.randint(0, cfg.freq_mask, size=(cfg.freq_mask_times, 2)):
        f0 = random.randrange(0, f - fw)
        if fw == 0:
            continue
        fmasks.append((f0, min(f0 + int(raw), f)))
    tmasks = []
    for tw, raw in np.random.randint(0, cfg.time_mask, size=(cfg.time_mask_times, 2)):
        if t - tw <= 0:
            continue
        t0 = random.randrange(0, t - tw)
        if tw == 0:
            continue
        tmasks.append((t0, min(t0 + int(raw), t)))
    return warp, fmasks, tmasks


def apply_plan(x, plan, replace_with_zero=False):
    x = np.array(x, dtype=np.float32, copy=True)
    warp, fmasks, tmasks = plan
    if warp is not None:
        center, warped = warp
        t = x.shape[0]
        left = resize_rows(x[:center], warped)
        right = resize_rows(x[center:], t - warped)
        x[:warped] = left
        x[warped:] = right
    for lo, hi in fmasks:
        x[:, lo:hi] = 0.0 if replace_with_zero else np.float32(x.astype(np.float64).mean())
    for lo, hi in tmasks:
        x[lo:hi] = 0.0 if replace_with_zero else np.float32(x.astype(np.float64).mean())
    return x
