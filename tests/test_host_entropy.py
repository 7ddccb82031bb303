"""Host entropy stage (no GPU): the batched boolean encoder in
image-webp_amd/csrc/zw_host_entropy.h is byte-identical to the reference's
bit-at-a-time ArithmeticEncoder (encoder/arithmetic.rs:7-196) over random
decision streams (skewed and uniform probabilities, long carry runs); the split
emission (recorded decisions, several frames' coders interleaved) is
byte-identical to the one-frame walk."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bool_encoder_batched_equals_reference(tmp_path):
    exe = str(tmp_path / "bool_equiv")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "image-webp_amd", "csrc"),
                           os.path.join(ROOT, "tools", "bool_equiv.cpp"), "-o", exe])
    out = subprocess.run([exe, "200000"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "equivalent" in out.stdout


def test_stats_token_paths_equal_reference_form(tmp_path):
    """record_coeffs via token paths == the reference's branchy record_coeffs
    (cost.rs:1297, never-cleared skip_eob), accumulated so the 0xfffe0000
    halving is exercised."""
    exe = str(tmp_path / "stats_equiv")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-I", os.path.join(ROOT, "image-webp_amd", "csrc"),
                           os.path.join(ROOT, "tools", "stats_equiv.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "equivalent" in out.stdout, out.stdout + out.stderr


def test_split_emission_equals_frame_walk(tmp_path):
    """zwh::emit_frames (K = 1..4 frames, decisions recorded per MB row, the
    frames' coders interleaved) == zwh::emit_frame on random packed records
    (every luma mode, skips, segments, sub-modes, all token categories, frame
    headers with and without probability updates), and the interleaved coder
    == the bit-at-a-time reference over random streams coded in pieces."""
    exe = str(tmp_path / "emit_equiv")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "image-webp_amd", "csrc"),
                           os.path.join(ROOT, "tools", "emit_equiv.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "equivalent" in out.stdout, out.stdout + out.stderr
