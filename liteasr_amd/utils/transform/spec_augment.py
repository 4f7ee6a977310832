"""SpecAugment (liteasr/utils/transform/spec_augment.py:14-125) on the device.

The reference augments each utterance on the CPU inside DataLoader workers (collator,
liteasr/dataset/asr_dataset.py:118): Pillow BICUBIC time warp, then ``freq_mask_times``
frequency masks and ``time_mask_times`` time masks filled with 0 or the running mean.

Here the work is split where it belongs on MI355X:

* the *random draws* stay on the host, in the same process and in exactly the reference's
  order -- ``random.randrange`` for the warp centre/width (:30-32), ``numpy.random.randint``
  for the mask sizes (:60-62, :93-95) and ``random.randrange`` for each mask start
  (:66, :100) -- so a seeded run consumes the two global RNG streams identically and draws
  the same numbers (``SpecAugment.plan``);
* the *pixels* are produced by one batched HIP call on the padded batch in HBM
  (csrc/specaug.hip, ``lasr_spec_augment``), bit-exact with Pillow for the warp.

``SpecAugment.__call__(x)`` keeps the reference's per-utterance interface (a (time, freq)
float32 tensor in, the augmented tensor out, same device); the training loader instead
draws one plan per utterance in the collator (``plan_batch``) and the trainer applies the
whole batch on the GPU after the host->device copy (``apply_batch``).  There is no CPU
fallback: without the native library every entry point raises.
"""

import random

import numpy as np
import torch

from . import register_transformation


@register_transformation("spec_aug")
class SpecAugment(object):
    device_capable = True

    def __init__(self, cfg):
        self.cfg = cfg

    @property
    def plan_stride(self):
        return 4 + 2 * (max(self.cfg.freq_mask_times, 0) + max(self.cfg.time_mask_times, 0))

    def plan(self, t, f):
        """Draw one utterance's random numbers (reference order); returns an int32 row."""
        cfg = self.cfg
        row = np.zeros(self.plan_stride, np.int32)
        window = cfg.time_warp
        if not (t - window <= window):  # time_warp :27-29
            center = random.randrange(window, t - window)
            warped = random.randrange(center - window, center + window) + 1
            row[0], row[1] = center, warped
        k = 4
        nf = 0
        for fw, raw in np.random.randint(0, cfg.freq_mask, size=(cfg.freq_mask_times, 2)):
            f0 = random.randrange(0, f - fw)
            if fw == 0:  # :68-70 (mask skipped, its start was still drawn)
                continue
            row[k], row[k + 1] = f0, min(f0 + int(raw), f)
            k += 2
            nf += 1
        nt = 0
        for tw, raw in np.random.randint(0, cfg.time_mask, size=(cfg.time_mask_times, 2)):
            if t - tw <= 0:  # :98-99 (no start drawn)
                continue
            t0 = random.randrange(0, t - tw)
            if tw == 0:
                continue
            row[k], row[k + 1] = t0, min(t0 + int(raw), t)
            k += 2
            nt += 1
        row[2], row[3] = nf, nt
        return row

    def plan_batch(self, lengths, f):
        """Plans for a minibatch, utterance by utterance in batch order: [B, plan_stride]."""
        out = np.zeros((len(lengths), self.plan_stride), np.int32)
        for i, t in enumerate(lengths):
            out[i] = self.plan(int(t), f)
        return torch.from_numpy(out)

    def apply_batch(self, xs, xlens, plan):
        """Augment a padded fp32 [B, T, F] device batch with precomputed plans."""
        from ... import kernels as K

        if not xs.is_cuda:
            raise RuntimeError("SpecAugment.apply_batch needs the batch on the GPU")
        B, T, _ = xs.shape
        if tuple(plan.shape) != (B, self.plan_stride):
            raise ValueError(f"plan shape {tuple(plan.shape)} != ({B}, {self.plan_stride})")
        # host-side validation of what the kernel indexes (the plan is host-built)
        p = plan.cpu() if plan.is_cuda else plan
        lens = xlens.cpu() if xlens.is_cuda else xlens
        if B and (int(lens.max()) > T or int(lens.min()) < 0):
            raise ValueError("xlens out of range for the padded batch")
        return K.spec_augment(xs.contiguous(), xlens.to(xs.device, torch.int64),
                              p.to(xs.device, torch.int32).contiguous(),
                              replace_with_zero=self.cfg.replace_with_zero)

    def __call__(self, x):
        """Reference interface: one (time, freq) tensor -> augmented tensor (same device)."""
        assert x.dim() == 2
        t, f = x.shape
        row = torch.from_numpy(self.plan(t, f)).unsqueeze(0)
        dev = x.device if x.is_cuda else torch.device("cuda")
        xs = x.to(dev, torch.float32).unsqueeze(0).contiguous()
        out = self.apply_batch(xs, torch.tensor([t], dtype=torch.int64, device=dev), row)
        return out[0].to(x.device)
