"""Drop-in for the reference's models/qnet.py (QNet + NoisyLinear, models/qnet.py:6-75).

Same constructor arguments, module tree, parameter/buffer names and shapes, so every reference
checkpoint (`torch.save` of state_dict()) loads unchanged, and the same reset_noise() semantics.

forward():
  * inference on a ROCm device (no autograd, 7 -> 3 net): the HIP path — the NoisyNet heads are
    folded on the device (mu, or mu + sigma*eps in train mode, qnet.py:43-50) and one
    pm_qnet_q launch evaluates the whole MLP + dueling combine;
  * a call that needs autograd (the reference's own train_step, train_iterative.py:152) keeps the
    reference's differentiable tensor semantics.
The batched learner never calls this module on its hot path; it runs the fused pm_selfplay_*
kernels on packed parameter blocks (pongmi.selfplay).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class NoisyLinear(nn.Module):
    def __init__(self, in_features, out_features, sigma_init=0.017):
        super().__init__()
        self.in_features = in_features
        self.out_features = out_features
        self.sigma_init = sigma_init
        self.weight_mu = nn.Parameter(torch.empty(out_features, in_features))
        self.bias_mu = nn.Parameter(torch.empty(out_features))
        self.weight_sigma = nn.Parameter(torch.empty(out_features, in_features))
        self.bias_sigma = nn.Parameter(torch.empty(out_features))
        self.register_buffer("weight_epsilon", torch.empty(out_features, in_features))
        self.register_buffer("bias_epsilon", torch.empty(out_features))
        self.reset_parameters()
        self.reset_noise()

    def reset_parameters(self):
        bound = 1.0 / math.sqrt(self.in_features)
        self.weight_mu.data.uniform_(-bound, bound)
        self.bias_mu.data.uniform_(-bound, bound)
        self.weight_sigma.data.fill_(self.sigma_init)
        self.bias_sigma.data.fill_(self.sigma_init)

    @staticmethod
    def _f(x):
        return x.sign().mul_(x.abs().sqrt_())

    def reset_noise(self):
        """Factorised Gaussian noise (models/qnet.py:33-41): eps_w = f(e_out) (x) f(e_in)."""
        dev = self.weight_mu.device
        e_in = self._f(torch.randn(self.in_features, device=dev))
        e_out = self._f(torch.randn(self.out_features, device=dev))
        self.weight_epsilon.copy_(e_out.ger(e_in))
        self.bias_epsilon.copy_(e_out)

    def effective(self):
        if self.training:
            return (self.weight_mu + self.weight_sigma * self.weight_epsilon,
                    self.bias_mu + self.bias_sigma * self.bias_epsilon)
        return self.weight_mu, self.bias_mu

    def forward(self, x):
        w, b = self.effective()
        return F.linear(x, w, b)


class QNet(nn.Module):
    def __init__(self, input_dim=7, output_dim=3):
        super().__init__()
        self.features = nn.Sequential(
            nn.Linear(input_dim, 64), nn.ReLU(),
            nn.Linear(64, 64), nn.ReLU(),
        )
        self.fc_V = NoisyLinear(64, 1)
        self.fc_A = NoisyLinear(64, output_dim)

    def reset_noise(self):
        for m in self.modules():
            if isinstance(m, NoisyLinear):
                m.reset_noise()

    def _device_path(self, x):
        return (x.is_cuda and x.dim() == 2 and x.shape[1] == 7 and self.fc_A.out_features == 3
                and self.features[0].in_features == 7
                and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())))

    def packed(self):
        """This net as a libpongmi parameter block [PM_QNET_NP] on its device."""
        from pongmi.qnet import PARAM_LAYOUT
        sd = self.state_dict()
        return torch.cat([sd[k].detach().reshape(-1).float() for k, _ in PARAM_LAYOUT])

    def forward(self, x):
        if self._device_path(x):
            from pongmi import _lib
            from pongmi.qnet import fold, q_values
            mode = _lib.PM_FOLD_TRAIN if self.training else _lib.PM_FOLD_EVAL
            return q_values(fold(self.packed(), mode)[0], x)
        h = self.features(x)
        V = self.fc_V(h)
        A = self.fc_A(h)
        return V + (A - A.mean(dim=1, keepdim=True))
