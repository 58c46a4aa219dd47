"""``LitModelGATsSPG`` for inference: the checkpoint wrapper ``inference.py:51-60`` loads.

The reference class (``src/models/GATsSPG_lightning_model.py:15-37``) is a Lightning module
holding a SuperPoint ``extractor``, the ``matcher`` and a focal-loss ``crit``; inference uses
only ``forward(x) -> self.matcher(x)`` after ``load_from_checkpoint(...).cuda().eval()
.freeze()``. Training, validation and the loss are out of scope, so this is
that inference surface over the HIP matcher: the same classmethod, the same ``forward``, the
same ``cuda`` / ``eval`` / ``freeze`` chain, the same checkpoint layout (``state_dict`` with
``matcher.*`` keys, flat ``hyper_parameters``).

The checkpoint is read with ``torch.load(weights_only=True)``: nothing in the file is
executed. Keys outside ``matcher.*`` (``extractor.*``, ``crit.*``) are ignored, as the
matcher never reads them.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .matcher import GATsSuperGlue, from_state_dict


def read_checkpoint(checkpoint_path: str):
    """(matcher state dict without the ``matcher.`` prefix, hyper-parameters dict or None)."""
    ckpt = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
    sd = ckpt.get("state_dict", ckpt)
    hp = ckpt.get("hyper_parameters")
    hp = dict(hp) if isinstance(hp, dict) else None
    if any(k.startswith("matcher.") for k in sd):
        sd = {k[len("matcher."):]: v for k, v in sd.items() if k.startswith("matcher.")}
    return sd, hp


def matcher_hparams(hparams):
    """The matcher's keys of a (flat) Lightning hyper-parameter dict over the GATsSPG
    defaults (``GATs_SuperGlue.py:166-201`` reads only these)."""
    from .synthetic import DEFAULT_HPARAMS
    if hparams is None:
        return dict(DEFAULT_HPARAMS)
    return {**DEFAULT_HPARAMS, **{k: hparams[k] for k in DEFAULT_HPARAMS if k in hparams},
            **({"attention_precision": hparams["attention_precision"]}
               if "attention_precision" in hparams else {})}


class LitModelGATsSPG(nn.Module):
    """Inference surface of ``GATsSPG_lightning_model.LitModelGATsSPG``."""

    def __init__(self, matcher: GATsSuperGlue, hparams=None):
        super().__init__()
        self.matcher = matcher
        self.hparams = dict(hparams or matcher.hparams)

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path: str, map_location=None, **overrides):
        """``LightningModule.load_from_checkpoint``: weights and hyper-parameters from the
        file; keyword arguments override hyper-parameters, as Lightning's do."""
        sd, hp = read_checkpoint(checkpoint_path)
        hp = {**(hp or {}), **overrides}
        m = cls(from_state_dict(sd, matcher_hparams(hp)), hp)
        if map_location is not None:
            m.to(map_location)
        return m

    def forward(self, x):
        return self.matcher(x)

    def freeze(self):
        """``LightningModule.freeze``: no gradients, eval mode."""
        for p in self.parameters():
            p.requires_grad = False
        return self.eval()
