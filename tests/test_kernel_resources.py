"""Register and scratch budgets of the band16 sweeps in the built library (no GPU needed): the
gfx950 code objects are read out of libgpx.so's fat binary (clang-offload-bundler) and their
kernel metadata (llvm-readelf --notes) checked against what the launch bounds promise —
DESIGN.md §3d: the Q <= 3 sweeps run two wavefronts per SIMD (<= 256 VGPRs), and no sweep the
C2 bench launches may spill to scratch (a spill turns the register-resident window into memory
traffic on every block step)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

from portfoliooptgp_amd import _native as N

LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
OBJCOPY = os.path.join(LLVM, "llvm-objcopy")
READELF = os.path.join(LLVM, "llvm-readelf")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _kernels():
    """{kernel symbol: (vgpr_count, agpr_count, private_segment_fixed_size)} over every TU."""
    if not (os.path.exists(N.LIB_PATH) and all(os.path.exists(t) for t in (BUNDLER, OBJCOPY, READELF))):
        pytest.skip("libgpx.so or the ROCm LLVM tools are absent")
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run([OBJCOPY, "--dump-section", f".hip_fatbin={fb}", N.LIB_PATH], check=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            chunk = os.path.join(d, f"b{i}")
            with open(chunk, "wb") as f:
                f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"b{i}.co")
            r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={chunk}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([READELF, "--notes", co], capture_output=True, text=True).stdout
            # one metadata map per kernel: fields in any order between "- " entries
            for block in re.split(r"\n\s+- \.", notes):
                m = re.search(r"\.?name:\s+(\S+)", block)
                if not m:
                    continue
                g = lambda k: int(re.search(k + r":\s+(\d+)", block).group(1)) if re.search(k + r":\s+(\d+)", block) else 0  # noqa: E731
                out[m.group(1)] = (g(r"\.vgpr_count"), g(r"agpr_count"), g(r"\.private_segment_fixed_size"))
    if not out:
        pytest.skip("no gfx950 code objects found in libgpx.so")
    return out


@pytest.fixture(scope="module")
def kernels():
    return _kernels()


def _find(kernels, pat):
    hits = {k: v for k, v in kernels.items() if re.search(pat, k)}
    assert hits, f"no kernel matches {pat}"
    return hits


# band16_fwd_kernel<Q, KIN>: _ZN3gpx17band16_fwd_kernelILi<Q>ELb<KIN>EEEv...
@pytest.mark.parametrize("q", [1, 2, 3])
def test_two_wave_sweeps_fit_256_registers(kernels, q):
    for name, (v, a, scratch) in _find(kernels, rf"band16_(fwd|fused)_kernelILi{q}E").items():
        assert v + a <= 256 and scratch == 0, (name, v, a, scratch)
    for name, (v, a, scratch) in _find(kernels, rf"band16_bwd_kernelILi{q}ELi1ELb1E").items():
        assert v + a <= 256 and scratch == 0, (name, v, a, scratch)


def test_bench_sweeps_do_not_spill(kernels):
    """Every sweep a C2 (SE1) evaluation can launch up to ℓ ≈ 2.4: band16 fwd/bwd for Q = 1..6
    with K's tiles computed in the sweeps (the default) or read from the K band, the fused sweeps,
    the wide (Q = 4/5, deferred) kernel, and the build."""
    pats = [r"band16_fwd_kernelILi[1-6]ELb[01]E", r"band16_bwd_kernelILi[1-6]ELi1ELb1ELb[01]E",
            r"band16_fused_kernelILi[1-5]ELb0ELb0E", r"band16_fused_kernelILi[1-5]ELb1ELb1E",
            r"band16_wide_kernelILb[01]ELb[01]ELi5E", r"band16_build_kernel"]
    for p in pats:
        for name, (v, a, scratch) in _find(kernels, p).items():
            # the two-wave Q = 4 inline-K backward (its W/P prefetch staged in LDS, Bwd16::LP)
            # keeps one 8-byte value in scratch across the step loop, reloaded after it
            budget = 16 if re.search(r"band16_bwd_kernelILi4ELi1ELb1ELb1E", name) else 0
            assert scratch <= budget, (name, v, a, scratch)


def test_two_wave_q4_backward(kernels):
    """The Q = 4 inline-K backward sweep runs two wavefronts per SIMD (<= 256 VGPRs + AGPRs)."""
    for name, (v, a, scratch) in _find(kernels, r"band16_bwd_kernelILi4ELi1ELb1ELb1E").items():
        assert v + a <= 256 and scratch <= 16, (name, v, a, scratch)


def test_widest_band16_classes_spill_within_budget(kernels):
    """Q = 7, 8 (ℓ ≈ 2.5-3.3 at the C2 inputs, SE1 with K inline): the window no longer fits the
    512 VGPRs + AGPRs of one wave; their spills stay under 1 KiB per lane (2 KiB for the wide
    launch that holds every class from 4 to 8), and nothing wider than Q = 8 is built."""
    for q in (7, 8):
        for name, (v, a, scratch) in _find(kernels, rf"band16_(fwd|bwd)_kernelILi{q}E").items():
            assert scratch <= 1024, (name, v, a, scratch)
    # the wide launch that also takes Q = 6..8 (one kernel: the widest branch sets its scratch)
    for name, (v, a, scratch) in _find(kernels, r"band16_wide_kernelILb1ELb1ELi8E").items():
        assert scratch <= 2048, (name, v, a, scratch)
    assert not [k for k in kernels if re.search(r"band16_(fwd|bwd)_kernelILi(9|1[0-9])E", k)]


def test_reduction_chain_and_call_kernels_do_not_spill(kernels):
    """The wide classes' reduction chain of block size 128 (round 6: bcrw_* and the bs = 128 build /
    contraction / finish — the latency route's Q = 6..8), the per-call reduce,
    the deferred part's input copy and result gather, and the fused small-problem kernel of the
    drop-in sizes (Np = 64): no scratch."""
    pats = [r"bcrw_fwd_factor_kernelILi8E", r"bcrw_fwd_delta_kernelILi8E", r"bcrw_bwd_kernelILi8E",
            r"bcr_build_kernelILi8E", r"bcr_contract_kernelILi8ELi[124]ELb1E", r"bcr_finish_kernel",
            r"reduce_kernel", r"slow_inputs_kernel", r"slow_gather_kernel", r"small64_kernel", r"small128_kernel", r"leaf128_kernel"]
    for p in pats:
        for name, (v, a, scratch) in _find(kernels, p).items():
            assert scratch == 0, (name, v, a, scratch)
            if p.startswith("bcrw") or "ILi8E" in p:
                assert v + a <= 256, (name, v, a)  # (8 waves per workgroup: two per SIMD)
