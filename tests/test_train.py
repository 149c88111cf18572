"""Optimizer (R13), schedules (N3), checkpoint format + resume (R16/R21),
the non-executing pickle reader, and the CPU plumbing end-to-end slice:
train -> save -> load -> sample -> SVG for both model families."""
import json
import math
import os
import pickle
import random

import numpy as np
import pytest
import torch

from sketch_rnn_amd.ckpt import checkpoint as ckpt
from sketch_rnn_amd.config import PRESETS, RefConfig, VAEConfig, load_json, save_json
from sketch_rnn_amd.train import schedules
from sketch_rnn_amd.train.optim import FlatAdam, adam_reference_step
from sketch_rnn_amd.utils import safe_pickle

REF_PKL = "/root/reference/save/kanji/config.pkl"


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(*s, generator=g)) for s in [(3, 5), (7,), (130,), (2, 2, 2)]]


@pytest.mark.parametrize("clip_mode,clip", [("global_norm", 0.5), ("global_norm", 1e9), ("value", 0.1), (None, 0.0)])
def test_flat_adam_matches_tf_adam(clip_mode, clip):
    ps = _params()
    ref = [p.detach().double().clone() for p in ps]
    ms = [torch.zeros_like(r) for r in ref]
    vs = [torch.zeros_like(r) for r in ref]
    opt = FlatAdam(ps, lr=0.01, eps=1e-3, clip_mode=clip_mode, clip=clip)
    assert opt.flat.numel() % 64 == 0
    g = torch.Generator().manual_seed(1)
    for t in range(1, 6):
        grads = [torch.randn(p.shape, generator=g) for p in ps]
        for p, gr in zip(ps, grads):
            p.grad.copy_(gr)
        opt.step()
        gd = [gr.double() for gr in grads]
        if clip_mode == "global_norm":
            norm = math.sqrt(sum(float((x * x).sum()) for x in gd))
            gd = [x * clip / max(norm, clip) for x in gd]
            assert abs(float(opt.scalars[2]) - norm) < 1e-4 * norm
        elif clip_mode == "value":
            gd = [x.clamp(-clip, clip) for x in gd]
        for k in range(len(ref)):
            ref[k], ms[k], vs[k] = adam_reference_step(ref[k], gd[k], ms[k], vs[k], t, 0.01, eps=1e-3)
    for p, r in zip(ps, ref):
        assert torch.allclose(p.detach().double(), r, atol=1e-5)
    assert int(opt.scalars[1]) == 5


def test_flat_adam_params_are_arena_views():
    ps = _params()
    opt = FlatAdam(ps, lr=0.1)
    with torch.no_grad():
        ps[1].fill_(3.0)
    o = opt.offsets[1]
    assert torch.all(opt.flat[o:o + 7] == 3.0)
    ps[2].grad.fill_(1.0)
    assert float(opt.grad.sum()) == 130.0
    opt.zero_grad()
    assert float(opt.grad.abs().sum()) == 0.0


def test_flat_adam_gather_grads_equals_accumulation():
    """zero_grad(set_to_none) + backward + gather_grads fills the arena
    exactly like accumulating into zeroed arena views; parameters without a
    gradient get zeroed slots (stale values from the previous step are
    cleared) and p.grad is rebound to the arena."""
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(5, 3)), torch.nn.Parameter(torch.randn(3)),
          torch.nn.Parameter(torch.randn(4))]
    x = torch.randn(7, 5)

    def loss():
        return ((x @ ps[0] + ps[1]) ** 2).sum()    # ps[2] unused

    opt = FlatAdam(ps, lr=0.1)
    opt.zero_grad()
    loss().backward()
    ref = opt.grad.clone()
    opt.grad.fill_(9.0)                              # stale contents
    opt.zero_grad(set_to_none=True)
    assert all(p.grad is None for p in ps)
    loss().backward()
    opt.gather_grads()
    o = opt.offsets
    for i, p in enumerate(ps):
        assert p.grad.data_ptr() == opt.grad[o[i]:].data_ptr()
        assert torch.equal(opt.grad[o[i]:o[i] + p.numel()], ref[o[i]:o[i] + p.numel()])
    assert float(opt.grad[o[2]:o[2] + 4].abs().sum()) == 0.0


def test_schedules():
    rc = RefConfig()
    assert schedules.reference_lr(rc, 0) == 0.005
    assert abs(schedules.reference_lr(rc, 10) - 0.005 * 0.99 ** 10) < 1e-15
    vc = VAEConfig()
    assert abs(schedules.vae_lr(vc, 0) - 0.001) < 1e-15
    assert abs(schedules.vae_lr(vc, 10 ** 7) - vc.min_learning_rate) < 1e-9
    assert abs(schedules.kl_weight(vc, 0) - vc.kl_weight_start) < 1e-15
    assert abs(schedules.kl_weight(vc, 10 ** 7) - vc.kl_weight) < 1e-9
    ws = [schedules.kl_weight(vc, s) for s in range(0, 50000, 5000)]
    assert all(a < b for a, b in zip(ws, ws[1:]))


def test_config_json_roundtrip_and_presets(tmp_path):
    for name, cfg in PRESETS.items():
        p = str(tmp_path / (name + ".json"))
        save_json(cfg, p)
        assert load_json(p) == cfg
    p = str(tmp_path / "ref.json")
    save_json(RefConfig(rnn_size=64), p)
    assert load_json(p) == RefConfig(rnn_size=64)
    assert PRESETS["vae_large"].dec_rnn_size == 2048 and PRESETS["vae_large"].dec_model == "hyper"
    assert PRESETS["vae_classcond"].num_classes == 345


@pytest.mark.skipif(not os.path.exists(REF_PKL), reason="reference tree not present")
def test_reference_config_pkl_safe_reader():
    cfg = RefConfig.from_config_pkl(REF_PKL)
    assert (cfg.rnn_size, cfg.num_layers, cfg.model, cfg.num_mixture, cfg.seq_length) == (256, 2, "lstm", 24, 300)
    assert cfg.dataset_name == "kanji" and cfg.data_scale == 15.0 and cfg.keep_prob == 0.8


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned > /dev/null",))


def test_safe_pickle_never_executes():
    data = pickle.dumps(_Evil(), protocol=2)
    obj = safe_pickle.loads(data)
    # the call is represented, never performed
    assert isinstance(obj, safe_pickle.Reconstructed)
    assert obj.callable.name == "system"
    ns = pickle.dumps({"a": 1, "b": [1.5, "x"], "c": (True, None)}, protocol=2)
    assert safe_pickle.loads(ns) == {"a": 1, "b": [1.5, "x"], "c": (True, None)}
    for proto in (0, 1, 2):
        assert safe_pickle.loads(pickle.dumps({"k": [1, 2.5, "s"]}, protocol=proto)) == {"k": [1, 2.5, "s"]}


def test_checkpoint_roundtrip_index_and_pruning(tmp_path):
    from sketch_rnn_amd.models.reference import SketchRNN
    cfg = RefConfig(rnn_size=16, num_mixture=3)
    m = SketchRNN(cfg, seed=0)
    opt = FlatAdam(m.parameters(), lr=0.01, eps=1e-3, clip_mode="global_norm", clip=5.0)
    for p in m.parameters():
        p.grad.normal_()
    opt.step()
    d = str(tmp_path / "save")
    for step in range(1, 8):
        ckpt.save_checkpoint(d, step, m, opt, cfg, extra={"epoch": step}, state={"s0": torch.ones(2, 3) * step},
                             keep=3)
    idx = open(os.path.join(d, "checkpoint")).read().splitlines()
    assert idx[0] == 'model_checkpoint_path: "model.ckpt-7"'
    assert idx[1:] == ['all_model_checkpoint_paths: "model.ckpt-%d"' % k for k in (5, 6, 7)]
    assert sorted(f for f in os.listdir(d) if f.endswith(".safetensors")) == \
        ["model.ckpt-%d.safetensors" % k for k in (5, 6, 7)]
    m2 = SketchRNN(cfg, seed=5)
    opt2 = FlatAdam(m2.parameters(), lr=0.5)
    step, extra, st = ckpt.load_checkpoint(ckpt.latest_checkpoint(d), m2, opt2)
    assert step == 7 and extra == {"epoch": 7} and torch.equal(st["s0"], torch.ones(2, 3) * 7)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)
    assert torch.equal(opt.m, opt2.m) and torch.equal(opt.v, opt2.v) and opt2.step_count == 1
    assert abs(opt2.lr - 0.01) < 1e-9
    assert ckpt.load_config(d) == cfg


def _ref_loader(n=40, seed=0):
    from sketch_rnn_amd.data.loader import SketchLoader
    from sketch_rnn_amd.data.synthetic import synthetic_reference_corpus
    return SketchLoader(4, 24, 15.0, sketches=synthetic_reference_corpus(n, seed=seed, max_len=40), seed=seed,
                        use_native=False)


def test_reference_plumbing_train_save_sample_svg(tmp_path):
    from sketch_rnn_amd.cli.sample import accept
    from sketch_rnn_amd.render.svg import draw_stroke_color_array
    from sketch_rnn_amd.sample.sampler import sample_reference
    from sketch_rnn_amd.train.trainer import ReferenceTrainer
    cfg = RefConfig(rnn_size=32, num_mixture=4, batch_size=4, seq_length=24, num_epochs=2, save_every=5,
                    dataset_name="synth")
    logs = []
    tr = ReferenceTrainer(cfg, _ref_loader(), save_root=str(tmp_path), log=logs.append,
                          metrics_path=str(tmp_path / "m.jsonl"))
    tr.train()
    assert tr.epoch == 2 and tr.b_processed > 4
    assert any("(epoch 0 batch 1), cost = " in l for l in logs)
    recs = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert len(recs) == tr.b_processed and all(math.isfinite(r["cost"]) for r in recs)
    from sketch_rnn_amd.cli.sample import load_model
    model = load_model(str(tmp_path / "synth"), "cpu")
    s, _ = sample_reference(model, 50, 0.5, 0.5, stop_if_eoc=True, rng=np.random.RandomState(0),
                            py_rng=random.Random(0))
    assert s.shape[1] == 5 and len(s) <= 50
    accept(s, 160.0)
    out = str(tmp_path / "o.svg")
    draw_stroke_color_array([s, s], svg_filename=out, block_size=160, maxcol=2)
    txt = open(out).read()
    assert txt.startswith("<?xml") and txt.count("<path") >= 2


def test_reference_resume_continues_epoch(tmp_path):
    from sketch_rnn_amd.train.trainer import ReferenceTrainer
    cfg = RefConfig(rnn_size=16, num_mixture=3, batch_size=4, seq_length=24, num_epochs=3, save_every=1000,
                    dataset_name="r")
    a = ReferenceTrainer(cfg, _ref_loader(), save_root=str(tmp_path / "a"), log=lambda s: None)
    a.train(max_batches=3)
    b = ReferenceTrainer(cfg, _ref_loader(), save_root=str(tmp_path / "a"), log=lambda s: None)
    assert b.resume()
    assert b.loader.pointer == a.loader.pointer and np.array_equal(b.loader.index, a.loader.index)
    # continuing both gives identical next batches and parameters
    a.train(max_batches=2)
    b.train(max_batches=2)
    for p, q in zip(a.model.parameters(), b.model.parameters()):
        assert torch.allclose(p, q, atol=1e-6)


def test_divergence_guard(tmp_path):
    from sketch_rnn_amd.train.trainer import DivergenceError, ReferenceTrainer
    cfg = RefConfig(rnn_size=16, num_mixture=3, batch_size=4, seq_length=24, divergence_bound=-1.0,
                    dataset_name="d")
    tr = ReferenceTrainer(cfg, _ref_loader(), save_root=str(tmp_path), log=lambda s: None)
    with pytest.raises(DivergenceError):
        tr.train(max_batches=2)


def _vae_sets(cfg, n=48):
    from sketch_rnn_amd.cli.vae_train import make_datasets
    return make_datasets(cfg, None, n)


def test_vae_plumbing_train_eval_resume_sample(tmp_path):
    from sketch_rnn_amd.data.strokes import to_normal_strokes
    from sketch_rnn_amd.render.svg import grid_strokes3
    from sketch_rnn_amd.sample.sampler import sample_vae
    from sketch_rnn_amd.train.trainer import VAETrainer
    cfg = VAEConfig(enc_rnn_size=16, dec_rnn_size=32, z_size=8, num_mixture=3, max_seq_len=40, batch_size=4,
                    dec_model="hyper", hyper_num_units=16, hyper_embedding_size=4, save_every=0, num_classes=2)
    (train, valid, test), scale = _vae_sets(cfg)
    logs = []
    tr = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "vae"), log=logs.append)
    tr.train(num_steps=6, log_every=3)
    assert tr.step == 6 and any(l.startswith("step: 6") for l in logs)
    ev = tr.evaluate(test)
    assert all(math.isfinite(v) for v in ev.values()) and ev["kl_cost"] >= cfg.kl_tolerance - 1e-6
    tr2 = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "vae"), log=logs.append)
    assert tr2.resume() and tr2.step == 6
    for p, q in zip(tr.model.parameters(), tr2.model.parameters()):
        assert torch.equal(p, q)
    assert tr2.evaluate(test) == ev
    s5, _ = sample_vae(tr2.model, 40, 0.5, rng=np.random.RandomState(0), label=1)
    s3 = to_normal_strokes(s5)
    grid_strokes3([s3, s3], str(tmp_path / "g.svg"))
    assert os.path.getsize(tmp_path / "g.svg") > 100


def test_cli_smoke(tmp_path):
    from sketch_rnn_amd.cli import preprocess as cp
    from sketch_rnn_amd.cli import sample as cs
    from sketch_rnn_amd.cli import train as ct
    from sketch_rnn_amd.cli import vae_sample as cvs
    from sketch_rnn_amd.cli import vae_train as cvt
    root = str(tmp_path)
    assert ct.main(["--synthetic", "30", "--rnn_size", "16", "--num_mixture", "3", "--batch_size", "4",
                    "--seq_length", "20", "--max_batches", "2", "--save_root", root, "--dataset_name", "s",
                    "--device", "cpu", "--no_graph"]) == 0
    assert cs.main(["--save_root", root, "--dataset_name", "s", "--num_picture", "1", "--sample_length", "30",
                    "--filename", root + "/out", "--device", "cpu", "--seed", "0", "--max_attempts", "3"]) == 0
    assert os.path.exists(root + "/out.svg")
    pk = root + "/p.skpack.npz"
    assert cp.main(["synthetic", pk, "--n", "40", "--classes", "2", "--max_len", "30"]) == 0
    assert cvt.main(["--data", pk, "--enc_rnn_size", "8", "--dec_rnn_size", "16", "--z_size", "4", "--num_mixture", "2",
                     "--batch_size", "4", "--max_seq_len", "30", "--num_steps", "2", "--save_dir", root + "/v",
                     "--device", "cpu", "--dtype", "fp32", "--no_graph", "--num_classes", "2"]) == 0
    assert cvs.main(["--save_dir", root + "/v", "--out", root + "/v.svg", "--n", "2", "--mode", "interpolate",
                     "--device", "cpu"]) == 0
    assert os.path.exists(root + "/v.svg")


def test_flat_adam_nonfinite_skip_and_apply():
    ps = _params()
    opt = FlatAdam(ps, lr=0.1, clip_mode="value", clip=1.0, nonfinite="skip")
    for p in ps:
        p.grad.fill_(0.5)
    opt.step()
    before = opt.flat.clone()
    m0 = opt.m.clone()
    ps[0].grad[0, 0] = float("nan")
    opt.step()
    assert torch.equal(opt.flat, before) and torch.equal(opt.m, m0)
    assert int(opt.scalars[1]) == 1 and opt.skipped_steps() == 1 and int(opt.scalars[4]) == 1
    ps[0].grad[0, 0] = 0.5
    opt.step()
    assert int(opt.scalars[1]) == 2 and int(opt.scalars[4]) == 0 and not torch.equal(opt.flat, before)
    ps2 = _params()
    opt2 = FlatAdam(ps2, lr=0.1, nonfinite="apply")
    for p in ps2:
        p.grad.fill_(0.5)
    ps2[1].grad[0] = float("inf")
    opt2.step()
    assert opt2.skipped_steps() == 0 and not torch.isfinite(opt2.flat).all()


def test_vae_metrics_jsonl_and_phases(tmp_path):
    from sketch_rnn_amd.train.trainer import VAETrainer
    from sketch_rnn_amd.utils.trace import PhaseTimes, phase
    cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=16, z_size=4, num_mixture=2, max_seq_len=24, batch_size=4,
                    save_every=0)
    (train, valid, test), _ = _vae_sets(cfg, n=40)
    m = str(tmp_path / "m.jsonl")
    tr = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "v"), log=lambda s: None, metrics_path=m)
    tr.train(num_steps=4, log_every=2)
    recs = [json.loads(l) for l in open(m)]
    assert [r["step"] for r in recs] == [2, 4]
    for r in recs:
        assert {"cost", "r_cost", "kl_cost", "grad_norm", "lr", "kl_weight", "strokes_per_s", "skipped",
                "host_ms"} <= set(r)
        assert "data" in r["host_ms"] and "step" in r["host_ms"] and r["skipped"] == 0
        # strokes_per_s counts valid (non-padding) points, like bench.py; positions_per_s the padded grid
        assert 0 < r["strokes_per_s"] < r["positions_per_s"]
    pt = PhaseTimes()
    with phase("x", pt):
        pass
    assert pt.count["x"] == 1 and "x" in pt.mean_ms()


def test_vae_training_reproducible_across_fresh_trainers(tmp_path):
    """Noise (dropout, reparameterisation eps) is keyed by (seed, step), not a
    process-global RNG: two fresh trainers in one process train identically."""
    from sketch_rnn_amd.train.trainer import VAETrainer
    cfg = VAEConfig(enc_rnn_size=16, dec_rnn_size=32, z_size=8, num_mixture=3, max_seq_len=30, batch_size=4,
                    dec_model="lstm", save_every=0)
    runs = []
    for k in range(2):
        (train, valid, test), _ = _vae_sets(cfg)
        tr = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / str(k)), log=lambda s: None)
        runs.append([float(tr.train_step(*tr.batch_to_device(train.random_batch()))["cost"]) for _ in range(3)])
        torch.randn(5)   # perturb the global RNG between runs
    assert runs[0] == runs[1]


def test_vae_resume_with_prefetch_is_exact(tmp_path):
    """Batches are produced ahead on a background thread; a checkpoint
    records the data state of the last batch consumed, so 3 steps + resume
    + 3 steps equals 6 uninterrupted steps bit for bit."""
    from sketch_rnn_amd.train.trainer import VAETrainer
    cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=16, z_size=4, num_mixture=2, max_seq_len=24, batch_size=4,
                    save_every=3)
    (train, valid, test), _ = _vae_sets(cfg)
    a = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "a"), log=lambda s: None)
    a.train(num_steps=6, log_every=3)
    (train, valid, test), _ = _vae_sets(cfg)
    b = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "b"), log=lambda s: None)
    b.train(num_steps=3, log_every=3)
    (train, valid, test), _ = _vae_sets(cfg)
    c = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "b"), log=lambda s: None)
    assert c.resume() and c.step == 3
    c.train(num_steps=6, log_every=3)
    assert torch.equal(a.opt.flat, c.opt.flat)


def test_vae_train_twice_continues_the_batch_sequence(tmp_path):
    """The prefetcher draws batches ahead; train() rewinds the dataset to the
    last batch consumed when it returns, so train(3); train(6) sees the same
    batches as one train(6) (checkpoint-free continuation)."""
    from sketch_rnn_amd.train.trainer import VAETrainer
    cfg = VAEConfig(enc_rnn_size=8, dec_rnn_size=16, z_size=4, num_mixture=2, max_seq_len=24, batch_size=4,
                    save_every=0)
    (train, valid, test), _ = _vae_sets(cfg)
    a = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "a"), log=lambda s: None)
    a.train(num_steps=6, log_every=3)
    (train, valid, test), _ = _vae_sets(cfg)
    b = VAETrainer(cfg, train, valid, test, save_dir=str(tmp_path / "b"), log=lambda s: None)
    b.train(num_steps=3, log_every=3)
    b.train(num_steps=6, log_every=3)
    assert torch.equal(a.opt.flat, b.opt.flat)


def test_fused_decoder_chunking_follows_cu_count():
    from sketch_rnn_amd.sample.fused import _chunk_rows
    assert _chunk_rows(2, 2) == (256 // 33) * 32
    assert _chunk_rows(2, 1, cus=80) == (80 // 33) * 16
    assert _chunk_rows(2, 1, cus=32) == 0      # -> NotCoResident, the CLI uses GraphDecoder


def test_grad_slot_only_when_unbound():
    from sketch_rnn_amd.ops import gemm
    from sketch_rnn_amd.train.optim import FlatAdam
    w = torch.nn.Parameter(torch.randn(4, 8))
    opt = FlatAdam([w], lr=0.1)
    assert gemm.grad_slot(w, (4, 8)) is None            # p.grad bound to the arena view
    opt.zero_grad(set_to_none=True)
    slot = gemm.grad_slot(w, (4, 8))
    assert slot is not None and slot.data_ptr() == opt.grad.data_ptr()
    assert gemm.grad_slot(w, (8, 4)) is None
