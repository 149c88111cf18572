"""Native libraries load on the host (no GPU needed) and the ctypes mirrors of
every kernel argument block match the compiled C++ layouts."""
import ctypes
import os
import sys

import pytest

from sketch_rnn_amd.utils import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hip():
    # (re)build when any csrc/*.hip is newer than the library; a no-op otherwise
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import build_native
    build_native.build_hip()
    lib = native.hip_lib()
    assert lib is not None
    return lib


def test_arg_struct_layouts(hip):
    from sketch_rnn_amd.ops import _hipapi as api
    for fn, cls in (("skr_lstm_fwd_args_size", api.LstmFwdArgs), ("skr_lstm_bwd_args_size", api.LstmBwdArgs),
                    ("skr_gru_fwd_args_size", api.GruFwdArgs), ("skr_gru_bwd_args_size", api.GruBwdArgs),
                    ("skr_lstm_fused_fwd_args_size", api.FusedFwdArgs),
                    ("skr_lstm_fused_bwd_args_size", api.FusedBwdArgs),
                    ("skr_gemm_problem_size", api.GemmProblem)):
        assert getattr(hip.lib, fn)() == ctypes.sizeof(cls), fn


def test_exported_entry_points(hip):
    for name in ("skr_lstm_fwd_step", "skr_lstm_bwd_step", "skr_gru_fwd", "skr_gru_bwd", "skr_skinny_gemm_v2",
                 "skr_skinny_gemm_v2", "skr_mdn_loss", "skr_adam_step", "skr_global_norm", "skr_mdn_sample",
                 "skr_lstm_fused_fwd", "skr_lstm_fused_bwd", "skr_colsum",
                 "skr_skinny_gemm_group"):
        assert hasattr(hip.lib, name), name


def test_host_packer_loads():
    if native.host_lib() is None:
        sys.path.insert(0, os.path.join(ROOT, "scripts"))
        import build_native
        build_native.build_host()
    assert native.host_lib() is not None


def test_host_packer_under_asan_ubsan(tmp_path):
    """the host runtime built with AddressSanitizer +
    UndefinedBehaviorSanitizer and driven over random corpora in its own
    process (host code only -- no GPU sanitizers on this pool)."""
    import shutil
    import subprocess
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "packer_sanitize")
    subprocess.check_call([gxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
                           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                           os.path.join(root, "csrc", "host", "tests", "packer_sanitize.cpp"),
                           os.path.join(root, "csrc", "host", "packer.cpp"), "-o", exe])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout
