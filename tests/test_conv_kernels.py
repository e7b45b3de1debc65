"""Op-level numerics of the 3x3 conv kernel family on the GPU (bf16 and IEEE-half storage, fp32
accumulate).

tools/convbench (built in-tree by __graft_entry__.build) runs every UNet 3x3 shape through each
kernel choice on random inputs and compares the full output with a naive one-thread-per-output
fp32 conv of the same bf16 operands and the same epilogue (bias, per-image scale/shift, SiLU,
residual): max |diff| / max |ref| < 1e-2; and, independently of any GPU code, 2048 sampled
outputs per shape against a host fp64 recomputation from the operands copied back ("host rel",
same bound). Choices: -1 built-in (conv3r register-stationary for 64 -> 64 on 256-pixel rows, v5
weight-stationary for 64 -> 64 on 128-pixel rows, swapped-epilogue v4 elsewhere), 70 conv3r, 18 v4
LDS epilogue, 40 / 41 swapped v4 256x64 / 128x64, 20 v4 128x64, 30 v5 without the SIMD-partner
offset, 0 v3."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tools", "convbench")


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["bf16", "f16"])
def test_conv3x3_kernels_match_naive_reference(dt):
    """Every 3x3 kernel choice on every UNet 3x3 shape, in bf16 and in IEEE half (CB_DTYPE=f16:
    the instantiations the fp16 headline runs), against the naive fp32 conv of the same
    16-bit operands and a host fp64 sample."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    env = dict(os.environ, CB_DTYPE=dt)
    out = subprocess.run([BIN, "1", "3x3", "check", "-1,70,18,40,41,20,30,0"], capture_output=True,
                         text=True, timeout=120, cwd=ROOT, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = [l for l in out.stdout.splitlines() if "check rel" in l]
    bad = [l for l in rows if not l.rstrip().endswith("OK")]
    assert len(rows) >= 40 and not bad, "\n".join(bad) or out.stdout[-2000:]
    # The shapes that take conv3r (variant 27: the three 256-wide 64 -> 64 shapes) and v5
    # (variant 21: the 128-wide one) by default really ran them.
    c3r = [l for l in rows if re.search(r"64->64 .*f-1\s+variant 27", l)]
    v5 = [l for l in rows if re.search(r"64->64 .*f-1\s+variant 21", l)]
    assert len(c3r) == 3 and len(v5) == 1, "\n".join(rows)


@pytest.mark.gpu
def test_norm_folded_gemms_match_host_reference():
    """SpatialTransformer norm1 -> q|k|v and norm3 -> GEGLU proj as ONE GEMM each (EPI_LNF: the
    LN gain folded into the weights, the row moments taken from the kernel's own A fragments,
    engine.cpp Packer::fold_ln) against a host fp64 LayerNorm + GEMM (+ GEGLU) with the exact
    weights, on rows offset by several standard deviations (attention.py:253-261; LN eps 1e-5);
    and proj_in with the GroupNorm(32, eps 1e-6) applied to its A fragments (EPI_GNA) against a
    host GroupNorm + GEMM (attention.py:76-77, 239-241). Bound 1e-2 max-rel: bf16 operands and
    output (measured figures in the printout)."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "lnf", "3"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = [l for l in out.stdout.splitlines() if "check" in l]
    assert len(rows) == 7 and all(l.rstrip().endswith("OK") for l in rows), out.stdout


@pytest.mark.gpu
def test_prenorm_layernorm_groupnorm_stats():
    """The SpatialTransformer's PreNorm LayerNorm kernel also produces the GroupNorm(32) statistics
    of its output (norm.hip layernorm_gnstats: per-block group sums, merged in fixed order by
    proj_in's table fill), so proj_in applies the GroupNorm in its A path with no
    separate pass (attention.py:76-77, 239-241). Against host fp64: xn rel < 1e-2 (bf16 output),
    GroupNorm mean abs < 1e-4 and rstd rel < 1e-4 from the merged block sums; run twice."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "gns"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = [l for l in out.stdout.splitlines() if "check" in l]
    assert len(rows) == 4 and all(l.rstrip().endswith("OK") for l in rows), out.stdout


@pytest.mark.gpu
def test_fp8_resblock_pair_matches_host_reference():
    """fp8 handles' ResBlock pair (conv3q.hip; module_util.py:143-153): block1's epilogue writes
    h as e4m3 with one E8M0 exponent per (pixel, 32 channels) — on the 64 -> 64 weight-stationary
    conv and on the fused-res_conv v4 tiles (64 | 64 concat input, whose 16-bit res_conv output
    must equal the 16-bit run's bit for bit) — and block2 runs on the block-scaled MFMA over it.
    Producer: every dequantized value within the e4m3 rounding of the 16-bit output (2^-4
    relative + 2^(e-8) absolute) and every exponent the smallest (+-1) with max / 2^e <= 448.
    Consumer: against a host fp64 conv of the dequantized operands with the same epilogue
    (bias, SiLU, + residual), max-rel < 1e-2 (bf16 output). Timing lines are printed."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "q8", "5"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = [l for l in out.stdout.splitlines() if "check" in l]
    assert len(rows) == 2 and all(l.rstrip().endswith("OK") for l in rows), out.stdout


@pytest.mark.gpu
def test_row_phase_upsample_conv_matches_plain():
    """The UNet's Upsample convs (nearest 2x then 3x3, module_util.py:100-103) in row-phase form
    (ConvArgs::uph: output row 2i+a reads source rows (i-1, i, i) or (i, i, i+1), so its kernel
    rows fold to (W0, W1+W2) / (W0+W1, W2) and each chunk takes 2 stages instead of 3) against
    the plain up conv with the same fp32 weights at the three UNet shapes, bf16 and IEEE half:
    max-rel < 1e-2 (the folded rows round to 16 bits once; measured ~5e-3 in bf16). Timing
    lines are printed."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "uph", "5"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = [l for l in out.stdout.splitlines() if "check" in l]
    assert len(rows) == 6 and all(l.rstrip().endswith("OK") for l in rows), out.stdout
    assert sum(l.startswith("f16") for l in rows) == 3, out.stdout


@pytest.mark.gpu
def test_fused_resblock_matches_conv3r_pair():
    """The 256x256 ResBlock as one launch (rbfuse.hip: block1 3x3 + scale/shift + SiLU, block2
    3x3 + SiLU + residual, Cin 128's 1x1 res_conv too; module_util.py:115-153) against the two
    conv3r launches it replaces, on random bf16 and IEEE-half data (9 cases each): bit-identical
    (same ordered MFMA sums and epilogue arithmetic) for one and two sources, ld2 != C2, B 1..8
    and Cin 64 / 128. Timing
    lines (pair vs fused) are printed; the engine takes the fused form only where it pays."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "rbf", "3"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    rows = [l for l in out.stdout.splitlines() if "check" in l]
    assert len(rows) == 18 and all(l.rstrip().endswith("check OK") for l in rows), out.stdout
    assert sum(l.startswith("f16") for l in rows) == 9, out.stdout


@pytest.mark.gpu
def test_small_grid_ring_depth_bit_identical():
    """The one-block-per-CU 3x3 v4 shapes (64x64 128->128, 32x32 256->256 at B = 8; module_util.py
    :111-153) run a 3-stage LDS ring by default (DAC_C3I_ST): a 2-, 3- and 4-stage ring must give
    bit-identical outputs (the stage count only buffers the same ordered MFMA sum)."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "st", "3"], capture_output=True, text=True, timeout=120, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "c3i st: OK" in out.stdout and "MISMATCH" not in out.stdout, out.stdout


@pytest.mark.gpu
def test_swapped_geglu_projection_bit_identical():
    """The SpatialTransformer's GEGLU projection (attention.py GEGLU: proj -> x * gelu(gate)) on
    swapped-operand tiles with the register epilogue (weights packed so each lane holds the x and
    gate accumulators of the same 8 output channels; engine.cpp Packer::geglu) against the
    LDS-epilogue tile on the same bf16 operands, at both UNet shapes (512 -> 2x2048 and
    256 -> 2x1024 on 32x32 x 8 images) and all four swapped tile sizes: bit-identical outputs
    (same ordered MFMA sums and epilogue arithmetic). Timing lines are printed."""
    assert os.path.exists(BIN), "tools/convbench missing: run __graft_entry__.build()"
    out = subprocess.run([BIN, "gsw", "5"], capture_output=True, text=True, timeout=120, cwd=ROOT)
    print(out.stdout)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    assert "gsw: OK" in out.stdout, out.stdout
    rels = [float(v) for v in re.findall(r"rel (\S+)", out.stdout)]
    assert len(rels) == 8 and all(v == 0.0 for v in rels), out.stdout
