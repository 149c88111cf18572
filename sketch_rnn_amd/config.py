"""Typed configuration.

Two configuration families:

* :class:`RefConfig` -- the reference decoder-only MDN-RNN. Field names and
  defaults are the reference's CLI flags (``train.py:14-43``), so a
  reference ``config.pkl`` maps onto it 1:1 (:func:`RefConfig.from_config_pkl`
  uses the non-executing reader in :mod:`.utils.safe_pickle`).
* :class:`VAEConfig` -- the seq2seq VAE (encoder / latent / decoder / MDN)
  with the sketch-rnn VAE hyper-parameter names.

Both serialize to JSON next to checkpoints. Framework-only knobs (precision,
kernel backend, graph capture, DP bucket size) live in :class:`RuntimeConfig`.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field, fields
from typing import Any, Dict


def _from_dict(cls, d: Dict[str, Any]):
    names = {f.name for f in fields(cls)}
    return cls(**{k: v for k, v in d.items() if k in names})


@dataclass
class RefConfig:
    """Reference decoder-only model flags (``train.py:14-43``)."""
    rnn_size: int = 256
    num_layers: int = 2
    model: str = "lstm"  # rnn | gru | lstm
    batch_size: int = 100
    seq_length: int = 300
    num_epochs: int = 500
    save_every: int = 250
    grad_clip: float = 5.0
    learning_rate: float = 0.005
    decay_rate: float = 0.99
    num_mixture: int = 24
    data_scale: float = 15.0
    keep_prob: float = 0.8
    stroke_importance_factor: float = 200.0
    dataset_name: str = "kanji"
    # framework additions (not in the reference)
    adam_eps: float = 1e-3        # model.py:183
    loss_clamp: float = 1e-20     # model.py:130
    divergence_bound: float = 30000.0  # train.py:94
    seed: int = 0

    kind: str = "reference"

    @property
    def n_out(self) -> int:
        return 3 + 6 * self.num_mixture

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d):
        return _from_dict(cls, d)

    @classmethod
    def from_config_pkl(cls, path: str) -> "RefConfig":
        from .utils.safe_pickle import load_namespace_pickle
        return cls.from_dict(load_namespace_pickle(path))


@dataclass
class VAEConfig:
    """seq2seq VAE hyper-parameters (sketch-rnn VAE names and defaults)."""
    data_set: str = "synthetic"
    num_steps: int = 10000000
    save_every: int = 500
    max_seq_len: int = 250
    dec_rnn_size: int = 512
    dec_model: str = "lstm"          # lstm | layer_norm | hyper
    enc_rnn_size: int = 256
    enc_model: str = "lstm"          # lstm | layer_norm
    z_size: int = 128
    kl_weight: float = 0.5
    kl_weight_start: float = 0.01
    kl_tolerance: float = 0.2
    batch_size: int = 100
    grad_clip: float = 1.0           # per-element clip_by_value
    num_mixture: int = 20
    learning_rate: float = 0.001
    decay_rate: float = 0.9999
    kl_decay_rate: float = 0.99995
    min_learning_rate: float = 0.00001
    use_recurrent_dropout: bool = True
    recurrent_dropout_prob: float = 0.90
    use_input_dropout: bool = False
    input_dropout_prob: float = 0.90
    use_output_dropout: bool = False
    output_dropout_prob: float = 0.90
    random_scale_factor: float = 0.15
    augment_stroke_prob: float = 0.10
    conditional: bool = True
    is_training: bool = True
    # HyperLSTM
    hyper_num_units: int = 256
    hyper_embedding_size: int = 32
    hyper_use_recurrent_dropout: bool = False
    hyper_use_layer_norm: bool = True   # LayerNorm main cell of the HyperLSTM (the hyper cell always has one)
    # class-conditional z (345 QuickDraw classes in the large config)
    num_classes: int = 0
    class_embed: str = "add"          # add | concat
    adam_eps: float = 1e-8
    seed: int = 0

    kind: str = "vae"

    @property
    def n_out(self) -> int:
        return 3 + 6 * self.num_mixture

    def to_dict(self):
        return dataclasses.asdict(self)

    @classmethod
    def from_dict(cls, d):
        return _from_dict(cls, d)

    def replace(self, **kw) -> "VAEConfig":
        return dataclasses.replace(self, **kw)


@dataclass
class RuntimeConfig:
    device: str = "cpu"
    dtype: str = "fp32"              # fp32 | bf16 (recurrent GEMM operand precision)
    backend: str = "auto"            # auto | hip | torch
    cuda_graph: bool = True          # capture the train step into a HIP graph
    dp_bucket_mb: float = 32.0
    log_every: int = 10


def save_json(cfg, path: str):
    with open(path, "w") as f:
        json.dump(cfg.to_dict(), f, indent=2, sort_keys=True)


def load_json(path: str):
    with open(path) as f:
        d = json.load(f)
    return (VAEConfig if d.get("kind") == "vae" else RefConfig).from_dict(d)


# named configs from BASELINE.json
PRESETS: Dict[str, VAEConfig] = {
    "plumbing": VAEConfig(conditional=False, dec_rnn_size=256, num_mixture=20),
    "vae_small": VAEConfig(enc_rnn_size=256, dec_rnn_size=512, dec_model="lstm"),
    "vae_large": VAEConfig(enc_rnn_size=512, dec_rnn_size=2048, dec_model="hyper"),
    "vae_classcond": VAEConfig(enc_rnn_size=512, dec_rnn_size=2048, dec_model="hyper", num_classes=345),
    "vae_layernorm": VAEConfig(enc_rnn_size=256, dec_rnn_size=512, dec_model="layer_norm"),
    "vae_layernorm_large": VAEConfig(enc_rnn_size=512, dec_rnn_size=2048, dec_model="layer_norm"),
}
