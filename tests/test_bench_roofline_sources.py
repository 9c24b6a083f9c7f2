"""bench.py's roofline traffic comes from the committed PMC summary of the kernel it names, on the
path the run takes: the inline-K summaries (*_kin3_*) when the library computes K's tiles in the
sweeps (its default, GPX_B16_INLINE_K unset or 3), the K-band ones otherwise."""
import os

import pytest

import bench


@pytest.mark.parametrize("key", ["band16_fwd_kernel", "band16_bwd_kernel", "band16_wide_kernel"])
def test_traffic_summary_follows_the_inline_k_setting(monkeypatch, key):
    monkeypatch.delenv("GPX_B16_INLINE_K", raising=False)
    t, src = bench.band_traffic(key, 10)
    assert src is not None and "_kin3_" in os.path.basename(src), src
    monkeypatch.setenv("GPX_B16_INLINE_K", "0")
    t0, src0 = bench.band_traffic(key, 10)
    assert src0 is not None and "_kin3_" not in os.path.basename(src0), src0
    assert t > 0 and t0 > t  # the K band through HBM costs bytes


def test_inline_k_traffic_is_within_five_megabytes_per_evaluation(monkeypatch):
    monkeypatch.delenv("GPX_B16_INLINE_K", raising=False)
    fwd, _ = bench.band_traffic("band16_fwd_kernel", 1)
    bwd, _ = bench.band_traffic("band16_bwd_kernel", 1)
    assert fwd + bwd <= 5e6, (fwd, bwd)
