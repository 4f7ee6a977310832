"""Transducer model restatement (encoder + LSTM prediction network + joint), CPU, fp32/fp64.

TEST INFRASTRUCTURE ONLY.  Only tests/ (and the golden generator) may import this module,
as the checker -- never as the thing measured or shipped.

Follows liteasr/models/transducer.py: forward :106-121 (h_enc.unsqueeze(2) + h_dec.unsqueeze(1)
through joint), joint :199-203 (lin_jnt(tanh(lin_enc(h_enc) + lin_dec(h_dec))), lin_dec without
bias :93), _preprocess :205-221 (ys_in = [blank | ys with -1 -> 0]); the prediction network
liteasr/nets/rnn_decoder.py:10-80 (nn.Embedding(padding_idx=0) -> n_layer LSTMCells, zero
initial state, torch's LSTMCell gate order i, f, g, o; dropout after the embedding and after
every cell).  The encoder is u2_oracle.encoder (transformer_encoder.py:107-127).  Pinned by
tests/test_oracle_golden.py against tests/golden/transducer.npz (the reference's own run)."""

from __future__ import annotations

import torch
import torch.nn.functional as F

from . import u2_oracle as O


def lstm_cell(x, h, c, p, name):
    """torch.nn.LSTMCell: gates = x W_ih^T + b_ih + h W_hh^T + b_hh -> (i, f, g, o)."""
    gates = F.linear(x, p[name + ".weight_ih"], p[name + ".bias_ih"]) + F.linear(h, p[name + ".weight_hh"],
                                                                                p[name + ".bias_hh"])
    i, f, g, o = gates.chunk(4, -1)
    i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
    c = f * c + i * g
    return o * torch.tanh(c), c


def prediction_network(ys_in, p, n_layer, units):
    """RNNDecoder.forward (rnn_decoder.py:69-80), dropout 0: (B, U+1) ids -> (B, U+1, units)."""
    y = F.embedding(ys_in, p["decoder.embed.weight"], padding_idx=0)  # no gradient into row 0
    B, U1 = ys_in.shape
    h = [torch.zeros(B, units, dtype=y.dtype) for _ in range(n_layer)]
    c = [torch.zeros(B, units, dtype=y.dtype) for _ in range(n_layer)]
    out = []
    for t in range(U1):
        x = y[:, t]
        for n in range(n_layer):
            h[n], c[n] = lstm_cell(x, h[n], c[n], p, f"decoder.dec_layers.{n}")
            x = h[n]
        out.append(x)
    return torch.stack(out, 1)


def decoder_input(ys, blank=0, ignore=-1):
    """Transducer._preprocess ys_in (transducer.py:211-214)."""
    return torch.cat([torch.full((ys.shape[0], 1), blank, dtype=ys.dtype), ys.masked_fill(ys == ignore, blank)], 1)


def joint(h_enc, h_dec, p):
    """Transducer.joint (transducer.py:199-203): h_enc (B, T, 1, d), h_dec (B, 1, U+1, units)."""
    e = F.linear(h_enc, p["lin_enc.weight"], p["lin_enc.bias"])
    dd = F.linear(h_dec, p["lin_dec.weight"])
    return F.linear(torch.tanh(e + dd), p["lin_jnt.weight"], p["lin_jnt.bias"])


def transducer_forward(xs, xlens, ys, ylens, p, cfg, bn_state=None, training=True):
    """Transducer.forward (transducer.py:106-121) -> (h_jnt (B, T', U+1, V), h_enc, h_dec)."""
    x, _ = O.encoder(xs, xlens, p, cfg, bn_state, training)
    h_dec = prediction_network(decoder_input(ys), p, cfg["dec_layers"], cfg["dec_units"])
    return joint(x.unsqueeze(2), h_dec.unsqueeze(1), p), x, h_dec
