"""f4: EODHD CSV → GP series (GPR/data_handler.py:26-90 semantics), against the oracle's
restatement used to build the golden fixtures."""
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
