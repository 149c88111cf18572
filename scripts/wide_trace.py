"""Per-step timeline of the wide persistent LN-LSTM forward (diagnostic).

Runs one forward of a [T, B, 2048] LayerNorm-LSTM with SKR_WIDE_TRACE=1 and
summarises the s_memrealtime stamps (100 MHz) every wave wrote (csrc/lstm_wide.hip,
``stamp``): CO waves 0..7 (0 loop top, 1 h_{t-1} arrived, 2 MFMA done,
3 gate tile published), RO waves 8..15 (0 loop top, 1 gate row arrived,
3 h_t published). Times in 10 ns ticks.
"""
import os
import sys

os.environ["SKR_WIDE_TRACE"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from sketch_rnn_amd import ops  # noqa: E402
from sketch_rnn_amd.ops import recurrent  # noqa: E402

T, B, H = int(os.environ.get("T", "40")), int(os.environ.get("B", "100")), 2048
ops.set_backend("hip")
ops.set_compute_dtype("bf16")
g = torch.Generator().manual_seed(0)
xp = (torch.randn(T, B, 4 * H, generator=g) * 0.5).cuda()
W = (torch.randn(H, 4 * H, generator=g) / H ** 0.5).cuda()
h0 = torch.zeros(B, H, device="cuda")
c0 = torch.zeros(B, H, device="cuda")
ln = (torch.ones(4 * H, device="cuda"), torch.zeros(4 * H, device="cuda"),
      torch.ones(H, device="cuda"), torch.zeros(H, device="cuda"))
with torch.no_grad():
    for _ in range(2):
        recurrent.WIDE_TRACES.clear()
        ops.lstm_sequence(xp, W, h0, c0, ln=ln)
        torch.cuda.synchronize()
tr = recurrent.WIDE_TRACES[-1].cpu().double()          # [T, NCO, 12, 4]
NCO = tr.shape[1]
nt = (B + 15) // 16
co = tr[:, :, :nt]                                       # CO waves in use
ro = tr[:, :, 8:16]
ro_on = ro[..., 3] > 0
t0 = co[0, :, :, 0][co[0, :, :, 0] > 0].min()
print("T=%d B=%d: whole launch %.1f us" % (T, B, (tr.max() - t0) / 100.0))
steps = []
for t in range(2, T - 1):
    c, r = co[t], ro[t][ro_on[t]]
    steps.append([
        c[..., 1].max() - c[..., 0].min(),                 # CO: first loop top -> last h arrival
        (c[..., 2] - c[..., 1]).mean(),                    # CO: MFMA phase (mean)
        (c[..., 2] - c[..., 1]).max(),                     # CO: MFMA phase (max)
        c[..., 3].max() - c[..., 2].min(),                 # CO: publish spread
        r[:, 1].max() - c[..., 3].max(),                   # hop CO publish -> RO arrival (last)
        (r[:, 3] - r[:, 1]).mean(),                        # RO: gather + LN + cell + publish (mean)
        (r[:, 3] - r[:, 1]).max(),                         # (max)
        co[t + 1][..., 1].max() - r[:, 3].max(),           # hop RO publish -> CO arrival (next step)
        co[t + 1][..., 1].max() - co[t][..., 1].max(),     # step period
    ])
s = torch.tensor(steps).mean(0)
names = ["CO wait spread", "CO mfma mean", "CO mfma max", "CO publish", "hop->RO", "RO work mean",
         "RO work max", "hop->CO", "STEP"]
for n, v in zip(names, s.tolist()):
    print("%-16s %8.1f ticks  (%.2f us)" % (n, v, v / 100.0))
