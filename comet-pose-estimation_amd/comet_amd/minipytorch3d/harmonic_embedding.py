"""HarmonicEmbedding (mirror of minipytorch3d/harmonic_embedding.py:14-185) on libcomet_hip.so
(comet_harmonic_fwd / comet_harmonic_bwd), same constructor and forward signature.
Not on COMET's live numeric path (SURVEY key finding 2), provided as the standalone operator."""
import torch

from .. import functional as F


class HarmonicEmbedding(torch.nn.Module):
    def __init__(self, n_harmonic_functions: int = 6, omega_0: float = 1.0, logspace: bool = True,
                 append_input: bool = True) -> None:
        super().__init__()
        if logspace:
            frequencies = 2.0 ** torch.arange(n_harmonic_functions, dtype=torch.float32)
        else:
            frequencies = torch.linspace(1.0, 2.0 ** (n_harmonic_functions - 1), n_harmonic_functions,
                                         dtype=torch.float32)
        self.register_buffer("_frequencies", frequencies * omega_0, persistent=False)
        self.register_buffer("_zero_half_pi", torch.tensor([0.0, 0.5 * torch.pi]), persistent=False)
        self.append_input = append_input

    def forward(self, x, diag_cov=None, **kwargs):
        return F.harmonic(x, self._frequencies, self.append_input, diag_cov)

    @staticmethod
    def get_output_dim_static(input_dims, n_harmonic_functions, append_input):
        return input_dims * (2 * n_harmonic_functions + int(append_input))

    def get_output_dim(self, input_dims=3):
        return self.get_output_dim_static(input_dims, len(self._frequencies), self.append_input)
