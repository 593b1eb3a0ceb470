"""NeRF positional encoding (mirror of scenedino/common/positional_encoding.py:44-90).

Keeps the reference's buffers (``_freqs``, ``_phases``) so state_dicts load
unchanged.  The fused gfx950 kernels compute the same 39-d code in registers; this
module's ``forward`` is the plain tensor-op form for API completeness.
"""
import numpy as np
import torch


class PositionalEncoding(torch.nn.Module):
    def __init__(self, num_freqs=6, d_in=3, freq_factor=np.pi, include_input=True):
        super().__init__()
        self.num_freqs = num_freqs
        self.d_in = d_in
        self.freqs = freq_factor * 2.0 ** torch.arange(0, num_freqs)
        self.d_out = self.num_freqs * 2 * d_in + (d_in if include_input else 0)
        self.include_input = include_input
        self.freq_factor = freq_factor
        self.register_buffer("_freqs", torch.repeat_interleave(self.freqs, 2).view(1, -1, 1))
        phases = torch.zeros(2 * self.num_freqs)
        phases[1::2] = np.pi * 0.5
        self.register_buffer("_phases", phases.view(1, -1, 1))

    def forward(self, x):
        embed = x.unsqueeze(1).repeat(1, self.num_freqs * 2, 1)
        embed = torch.sin(torch.addcmul(self._phases, embed, self._freqs)).view(x.shape[0], -1)
        return torch.cat((x, embed), dim=-1) if self.include_input else embed

    @classmethod
    def from_conf(cls, conf, d_in=3):
        return cls(conf.get("num_freqs", 6), d_in, conf.get("freq_factor", np.pi),
                   conf.get("include_input", True))
