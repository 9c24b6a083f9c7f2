"""f4: EODHD CSV → GP series (GPR/data_handler.py:26-90 semantics), against the oracle's
restatement used to build the golden fixtures."""
import os

import numpy as np
import pandas as pd
import pytest

from oracle import gp_oracle as O
from portfoliooptgp_amd import data


def _csv(tmp_path, n=40, seed=0):
    rng = np.random.default_rng(seed)
    dates = pd.bdate_range("2024-02-01", periods=n)
    close = 100 * np.exp(np.cumsum(rng.standard_normal(n) * 0.01))
    open_ = close * (1 + rng.standard_normal(n) * 0.003)
    df = pd.DataFrame(dict(date=dates.strftime("%Y-%m-%d"), open=open_, high=close * 1.01, low=close * 0.99,
                           close=close, adjusted_close=close, volume=rng.integers(1e5, 1e6, n)))
    p = tmp_path / f"T{seed}_us_d.csv"
    df.to_csv(p, index=False)
    return str(p)


def test_process_csv_matches_oracle_restatement(tmp_path):
    for seed in range(3):
        p = _csv(tmp_path, 30 + 7 * seed, seed)
        for col in ("return", "intraday_return"):
            X, Y, dates, mean, std = data.process_csv(p, "2024-02-01", col)
            xo, yo, mo, so = O.prepare_series(p, "2024-02-01", col)
            np.testing.assert_array_equal(X.numpy(), xo)
            np.testing.assert_array_equal(Y.numpy(), yo)
            assert (mean, std) == (mo, so)
    series, meta = data.load_series([_csv(tmp_path, 20, 9), _csv(tmp_path, 25, 10)], "2024-01-01")
    assert [len(x) for x, _ in series] == [20, 25] and meta[1]["path"].endswith("T10_us_d.csv")


def test_future_inputs_periods(tmp_path):
    p = _csv(tmp_path, 10, 4)
    last = pd.to_datetime(pd.read_csv(p)["date"]).max()
    xd = data.future_inputs(p, "2024-02-01", "d", 90).numpy()[:, 0]
    assert len(xd) == 90 and xd[0] == (last - pd.Timestamp("2024-02-01")).days + 1
    assert np.all(np.diff(xd) == 1)
    assert len(data.future_inputs(p, "2024-02-01", "w", 90)) == 12
    assert len(data.future_inputs(p, "2024-02-01", "m", 90)) == 3
    with pytest.raises(ValueError):
        data.future_inputs(p, "2024-02-01", "q")


INVESTING = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "investing")


@pytest.mark.parametrize("name", ["RUT2000", "DJI", "NasDaq100"])
def test_convert_investing_csv_reproduces_reference_files(name, tmp_path):
    """handle.py:38-75 (convert_csv + sort_csv) on the reference's own investing.com exports
    reproduces the converted files the reference keeps beside them, byte for byte (DJI carries
    quoted thousands separators, RUT2000 empty volumes, NasDaq100 'M' volume suffixes)."""
    out = tmp_path / f"{name}_us_d.csv"
    text = data.convert_investing_csv(os.path.join(INVESTING, f"{name}.csv"), str(out))
    with open(os.path.join(INVESTING, f"{name}_us_d.csv"), newline="") as f:
        ref = f.read()
    assert text == ref
    with open(out, newline="") as f:
        assert f.read() == ref


def test_load_batch_matches_process_csv(tmp_path):
    paths = [_csv(tmp_path, 20 + 3 * s, 20 + s) for s in range(5)]
    series, meta = data.load_batch(paths, "2024-01-15", "intraday_return", device=None, workers=3)
    for p, (X, Y), m in zip(paths, series, meta):
        Xr, Yr, dates, mean, std = data.process_csv(p, "2024-01-15", "intraday_return")
        assert X.shape == Xr.shape and Y.shape == Yr.shape
        np.testing.assert_array_equal(X.numpy(), Xr.numpy())
        np.testing.assert_array_equal(Y.numpy(), Yr.numpy())
        assert (m["mean"], m["std"], m["n"], m["path"]) == (mean, std, len(Xr), p)
        assert X.is_contiguous() and Y.is_contiguous()
