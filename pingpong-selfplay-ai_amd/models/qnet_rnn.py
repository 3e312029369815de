"""Drop-in for the reference's models/qnet_rnn.py (QNetRNN + NoisyLinear, models/qnet_rnn.py:8-152).

Same constructor arguments, module tree, parameter/buffer names and shapes, so the reference's
checkpoints (checkpoints_rnn/*.pth, modelB_state / modelA_state) load unchanged, and the same
forward(x_sequence, (h, c)) -> (q, (h_n, c_n)) / init_hidden / reset_noise contract.

forward():
  * inference on a ROCm device for the default shape (7 -> 64 -> 128, one 128-unit LSTM layer,
    128-unit shared head, 3 actions) with no autograd: the HIP path — NoisyLinear folded on the
    device (mu, or mu + sigma*eps in train mode, :43-50) and one pm_rnn_q launch per time step
    for the whole batch (features, LSTM cell, heads and dueling combine fused);
  * anything else (autograd, other shapes, CPU) keeps the reference's tensor semantics.
"""
import torch
import torch.nn as nn

from .qnet import NoisyLinear

__all__ = ["NoisyLinear", "QNetRNN"]


class QNetRNN(nn.Module):
    def __init__(self, input_dim=7, output_dim=3, feature_dim=128, lstm_hidden_dim=128, lstm_layers=1,
                 head_hidden_dim=128):
        super().__init__()
        self.input_dim = input_dim
        self.feature_dim = feature_dim
        self.lstm_hidden_dim = lstm_hidden_dim
        self.lstm_layers = lstm_layers
        self.head_hidden_dim = head_hidden_dim
        self.features_extractor = nn.Sequential(
            nn.Linear(input_dim, feature_dim // 2), nn.ReLU(),
            nn.Linear(feature_dim // 2, feature_dim), nn.ReLU(),
        )
        self.lstm = nn.LSTM(input_size=feature_dim, hidden_size=lstm_hidden_dim, num_layers=lstm_layers,
                            batch_first=True)
        if head_hidden_dim > 0:
            self.fc_shared_head = nn.Sequential(NoisyLinear(lstm_hidden_dim, head_hidden_dim), nn.ReLU())
            head_in = head_hidden_dim
        else:
            self.fc_shared_head = None
            head_in = lstm_hidden_dim
        self.fc_V = NoisyLinear(head_in, 1)
        self.fc_A = NoisyLinear(head_in, output_dim)

    def reset_noise(self):
        for m in self.modules():
            if isinstance(m, NoisyLinear):
                m.reset_noise()

    def init_hidden(self, batch_size, device):
        z = torch.zeros(self.lstm_layers, batch_size, self.lstm_hidden_dim, device=device)
        return z, z.clone()

    def _default_shape(self):
        return (self.input_dim == 7 and self.feature_dim == 128 and self.lstm_hidden_dim == 128
                and self.lstm_layers == 1 and self.head_hidden_dim == 128 and self.fc_A.out_features == 3)

    def _device_path(self, x):
        return (x.is_cuda and x.dim() == 3 and x.shape[2] == 7 and x.shape[1] >= 1 and self._default_shape()
                and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())))

    def packed(self):
        """This net as a libpongmi parameter block [PM_RNN_NP] on its device."""
        from pongmi.rnn import PARAM_LAYOUT
        sd = self.state_dict()
        return torch.cat([sd[k].detach().reshape(-1).float() for k, _ in PARAM_LAYOUT])

    def forward(self, x_sequence, hidden_state_tuple):
        if self._device_path(x_sequence):
            from pongmi import _lib
            from pongmi import rnn
            mode = _lib.PM_FOLD_TRAIN if self.training else _lib.PM_FOLD_EVAL
            B = x_sequence.shape[0]
            h0, c0 = hidden_state_tuple
            q, h, c = rnn.forward(rnn.fold(self.packed(), mode)[0], x_sequence, h0.reshape(B, -1),
                                  c0.reshape(B, -1))
            return q, (h.unsqueeze(0), c.unsqueeze(0))
        B, T, _ = x_sequence.shape
        feats = self.features_extractor(x_sequence.reshape(B * T, self.input_dim)).reshape(B, T, self.feature_dim)
        out, (h_n, c_n) = self.lstm(feats, hidden_state_tuple)
        x = out[:, -1, :]
        if self.fc_shared_head is not None:
            x = self.fc_shared_head(x)
        V = self.fc_V(x)
        A = self.fc_A(x)
        return V + (A - A.mean(dim=1, keepdim=True)), (h_n, c_n)
