"""Mixture-density head: parameterization, loss, sampling math.

Column layout of the head output ``z [N, 3 + 6M]`` (reference
``model.py:142-163``; identical in the sketch-rnn VAE):
``[pen(3) | pi(M) | mu1(M) | mu2(M) | sigma1_hat(M) | sigma2_hat(M) | rho_hat(M)]``
with ``pi = softmax``, ``sigma = exp``, ``rho = tanh``.

Two loss semantics (``mode``):

* ``"reference"`` (``model.py:124-139``): ``L_shape = mean(-log(max(S, 1e-20)))``
  over every step (no mask, rows are packed), ``L_pen = mean(w * CE)`` with
  ``w = cont + sqrt(F) eos + F eoc``; targets ``[dx, dy, eos, eoc, cont]``.
* ``"magenta"``: ``L_r = mean(fs * -log(S + 1e-6) + CE [* fs when eval])``
  with ``fs = 1 - p3`` (the end-of-sketch mask); targets ``[dx, dy, p1, p2, p3]``.

``S = sum_k pi_k N(x | mu_k, sigma_k, rho_k)`` is evaluated in log space
(``logsumexp``) so that it cannot underflow; the reference's clamp is kept
exactly: when ``S < 1e-20`` the shape term is ``-log(1e-20)`` with zero
gradient (``tf.maximum`` routes the gradient to the constant).
"""
from __future__ import annotations

import math
from typing import Tuple

import torch
import torch.nn.functional as F

LOG_2PI = math.log(2.0 * math.pi)


def split_z(z: torch.Tensor, M: int):
    pen = z[..., 0:3]
    pi, mu1, mu2, s1, s2, rho = torch.split(z[..., 3:3 + 6 * M], M, dim=-1)
    return pen, pi, mu1, mu2, s1, s2, rho


def mixture_coef(z: torch.Tensor, M: int):
    """``(pi, mu1, mu2, sigma1, sigma2, rho, pen_prob, pen_logits)``."""
    pen, pi, mu1, mu2, s1, s2, rho = split_z(z, M)
    return (torch.softmax(pi, -1), mu1, mu2, torch.exp(s1), torch.exp(s2), torch.tanh(rho),
            torch.softmax(pen, -1), pen)


def log_bivariate_normal(x1, x2, mu1, mu2, log_s1, log_s2, rho_hat):
    """log N(x | mu, sigma, rho) from the *raw* head outputs (Graves eq. 24-25)."""
    s1, s2, rho = torch.exp(log_s1), torch.exp(log_s2), torch.tanh(rho_hat)
    n1 = (x1 - mu1) / s1
    n2 = (x2 - mu2) / s2
    om = 1.0 - rho * rho
    zz = n1 * n1 + n2 * n2 - 2.0 * rho * n1 * n2
    return -zz / (2.0 * om) - LOG_2PI - log_s1 - log_s2 - 0.5 * torch.log(om)


def log_mixture_density(z: torch.Tensor, x1: torch.Tensor, x2: torch.Tensor, M: int) -> torch.Tensor:
    _, pi, mu1, mu2, s1, s2, rho = split_z(z, M)
    lp = torch.log_softmax(pi, -1) + log_bivariate_normal(x1.unsqueeze(-1), x2.unsqueeze(-1), mu1, mu2, s1, s2, rho)
    return torch.logsumexp(lp, -1)


def mdn_loss_torch(z: torch.Tensor, target: torch.Tensor, M: int, mode: str = "magenta",
                   stroke_importance: float = 200.0, is_training: bool = True,
                   clamp: float = 1e-20, eps: float = 1e-6) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Returns ``(total, shape_term, pen_term)`` (each a mean over rows)."""
    z = z.reshape(-1, z.shape[-1])
    if z.dtype != torch.float64:
        z = z.float()  # low-precision head outputs: the loss math runs in fp32
    target = target.reshape(-1, 5).to(z.dtype)
    x1, x2, pen_t = target[:, 0], target[:, 1], target[:, 2:5]
    logS = log_mixture_density(z, x1, x2, M)
    ce = -(pen_t * torch.log_softmax(z[:, 0:3], -1)).sum(-1)
    if mode == "reference":
        log_clamp = math.log(clamp)
        shape = torch.where(logS < log_clamp, torch.full_like(logS, -log_clamp), -logS)
        w = pen_t[:, 2] + math.sqrt(stroke_importance) * pen_t[:, 0] + stroke_importance * pen_t[:, 1]
        pen = w * ce
    elif mode == "magenta":
        fs = 1.0 - pen_t[:, 2]
        # -log(S + eps) = -logaddexp(log S, log eps)
        shape = -torch.logaddexp(logS, torch.full_like(logS, math.log(eps))) * fs
        pen = ce * fs if not is_training else ce
    else:
        raise ValueError(mode)
    s, p = shape.mean(), pen.mean()
    return s + p, s, p


def mdn_loss_prob_space(z: torch.Tensor, target: torch.Tensor, M: int, stroke_importance: float = 200.0):
    """Literal transcription of the reference math in probability space
    (``model.py:112-139``), used only to check :func:`mdn_loss_torch`."""
    z = z.reshape(-1, z.shape[-1]).double()
    t = target.reshape(-1, 5).double()
    pi, mu1, mu2, s1, s2, rho, _, pen_logits = mixture_coef(z, M)
    x1, x2 = t[:, 0:1], t[:, 1:2]
    n1, n2 = x1 - mu1, x2 - mu2
    s1s2 = s1 * s2
    zz = (n1 / s1) ** 2 + (n2 / s2) ** 2 - 2 * rho * n1 * n2 / s1s2
    neg_rho = 1 - rho ** 2
    res = torch.exp(-zz / (2 * neg_rho)) / (2 * math.pi * s1s2 * torch.sqrt(neg_rho))
    res1 = -torch.log(torch.clamp((res * pi).sum(1, keepdim=True), min=1e-20))
    shape = res1.mean()
    pen_data = t[:, 2:5]
    ce = -(pen_data * torch.log_softmax(pen_logits, -1)).sum(-1)
    w = pen_data[:, 2] + math.sqrt(stroke_importance) * pen_data[:, 0] + stroke_importance * pen_data[:, 1]
    pen = (ce * w).mean()
    return shape + pen, shape, pen
