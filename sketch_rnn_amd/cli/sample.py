"""``python -m sketch_rnn_amd.cli.sample`` -- reference sampling CLI (``sample.py:16-111``).

Loads ``save/<dataset>/config.json`` (or a reference ``config.pkl`` through
the non-executing pickle reader) and the latest checkpoint, then generates
``num_picture`` sketches with the reference rejection filter (stroke count
in ``[4, 22]``, at least one ``eoc``, bounding box within
``[0, 0.8] * picture_size``) and writes a colour SVG grid.

``--device_sampler`` draws candidates in parallel batches on the GPU
instead of the one-stroke-at-a-time host loop: with the fused whole-sketch
decoder (``sample.fused.FusedRefDecoder``, one kernel launch per batch)
when the model is eligible (2 x 256 LSTM class), otherwise with the
HIP-graph decoder (``sample.sampler.GraphDecoder``; ``--graph_decoder``
forces it).
"""
from __future__ import annotations

import argparse
import os
import random
import sys

import numpy as np


def build_parser():
    p = argparse.ArgumentParser(description="sample sketches from a trained sketch-rnn model")
    p.add_argument("--filename", type=str, default="output", help="filename of .svg file to output, without .svg")
    p.add_argument("--sample_length", type=int, default=600, help="number of strokes to sample")
    p.add_argument("--picture_size", type=float, default=160, help="a centered svg will be generated of this size")
    p.add_argument("--scale_factor", type=float, default=1,
                   help="factor to scale down by for svg output.  smaller means bigger output")
    p.add_argument("--num_picture", type=int, default=20, help="number of pictures to generate")
    p.add_argument("--num_col", type=int, default=5, help="if num_picture > 1, how many pictures per row?")
    p.add_argument("--dataset_name", type=str, default="kanji", help="name of directory containing training data")
    p.add_argument("--color_mode", type=int, default=1, help="set to 0 if you are a black and white sort of person...")
    p.add_argument("--stroke_width", type=float, default=2.0, help="thickness of pen lines")
    p.add_argument("--temperature", type=float, default=0.1, help="sampling temperature")
    # framework additions
    p.add_argument("--save_root", type=str, default="save")
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--seed", type=int, default=None)
    p.add_argument("--device_sampler", action="store_true")
    p.add_argument("--graph_decoder", action="store_true",
                   help="with --device_sampler: per-stroke HIP-graph decoder instead of the fused one-launch decoder")
    p.add_argument("--batch", type=int, default=64, help="candidates per device-sampler replay")
    p.add_argument("--max_attempts", type=int, default=100000)
    p.add_argument("--fix_pen_temperature", action="store_true")
    return p


def accept(strokes: np.ndarray, frame: float, min_size_ratio=0.0, max_size_ratio=0.8, min_num_stroke=4,
           max_num_stroke=22) -> bool:
    """Reference rejection filter (``sample.py:69-95``)."""
    from ..render.svg import calculate_start_point
    _, _, num_stroke, num_char, _ = strokes.sum(0)
    if num_stroke < min_num_stroke or num_char == 0 or num_stroke > max_num_stroke:
        return False
    _, _, sx, sy = calculate_start_point(strokes)
    if sx > frame * max_size_ratio or sy > frame * max_size_ratio:
        return False
    if sx < frame * min_size_ratio or sy < frame * min_size_ratio:
        return False
    return True


def load_model(save_dir: str, device: str):
    import torch
    from ..ckpt import checkpoint as ckpt
    from ..config import RefConfig, load_json
    from ..models.reference import SketchRNN
    if os.path.exists(os.path.join(save_dir, "config.json")):
        cfg = load_json(os.path.join(save_dir, "config.json"))
    else:
        cfg = RefConfig.from_config_pkl(os.path.join(save_dir, "config.pkl"))
    model = SketchRNN(cfg).to(device)
    path = ckpt.latest_checkpoint(save_dir)
    if path is None:
        raise FileNotFoundError("no checkpoint in %s" % save_dir)
    print("loading model: ", path)
    ckpt.load_checkpoint(path, model)
    model.eval()
    return model


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    import torch
    from ..render.svg import draw_stroke_color_array
    from ..sample.sampler import GraphDecoder, sample_reference
    device = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    model = load_model(os.path.join(a.save_root, a.dataset_name), device)
    rng = np.random.RandomState(a.seed)
    py_rng = random.Random(a.seed)
    accepted, attempts = [], 0
    if a.device_sampler and device.startswith("cuda"):
        from ..sample.fused import FusedRefDecoder, NotCoResident, fused_decode_ok

        def graph_decoder():
            return GraphDecoder(model, a.batch, a.sample_length, a.temperature,
                                fix_pen_temperature=a.fix_pen_temperature)
        dec = None
        if fused_decode_ok(model) and not a.graph_decoder:   # one launch per batch (csrc/decode_ref.hip)
            try:
                dec = FusedRefDecoder(model, a.batch, a.sample_length, a.temperature,
                                      fix_pen_temperature=a.fix_pen_temperature)
            except NotCoResident as e:
                print("fused decoder unavailable (%s); using the graph decoder" % e)
        if dec is None:
            dec = graph_decoder()
        while len(accepted) < a.num_picture and attempts < a.max_attempts:
            seed = rng.randint(1 << 30)
            try:
                strokes, lengths = dec.run(seed=seed)
            except NotCoResident as e:           # a smaller device than the chunking assumed
                print("fused decoder unavailable (%s); using the graph decoder" % e)
                dec = graph_decoder()
                strokes, lengths = dec.run(seed=seed)
            s_np, l_np = strokes.cpu().numpy(), lengths.cpu().numpy()
            for k in range(a.batch):
                attempts += 1
                s = s_np[k, : l_np[k]]
                if accept(s, a.picture_size) and len(accepted) < a.num_picture:
                    accepted.append(s)
                    print(len(accepted), "/", a.num_picture)
    else:
        while len(accepted) < a.num_picture and attempts < a.max_attempts:
            attempts += 1
            print(".", end="", flush=True)
            s, _ = sample_reference(model, a.sample_length, a.temperature, a.temperature, stop_if_eoc=True, rng=rng,
                                    py_rng=py_rng, fix_pen_temperature=a.fix_pen_temperature)
            if accept(s, a.picture_size):
                accepted.append(s)
                print(len(accepted), "/", a.num_picture)
    draw_stroke_color_array(accepted, factor=a.scale_factor, svg_filename=a.filename + ".svg",
                            stroke_width=a.stroke_width, block_size=a.picture_size, maxcol=a.num_col,
                            color_mode=a.color_mode != 0, rng=py_rng)
    print("wrote %s.svg (%d sketches, %d attempts)" % (a.filename, len(accepted), attempts))
    return 0


if __name__ == "__main__":
    sys.exit(main())
