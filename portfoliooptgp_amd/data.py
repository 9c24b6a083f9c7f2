"""On-disk input format → device-ready series.

The reference reads EODHD end-of-day CSVs (``date,open,high,low,close,adjusted_close,volume``,
e.g. ``Stocks/AAPL_EOD/AAPL_us_d.csv``) and turns each into a GP training set in
``GPR/data_handler.py:26-65``: X = days since ``train_start_date`` (unnormalised), Y = the
z-scored (pandas ddof=1) ``return`` = ``close.pct_change()`` with row 0 filled by row 1's
return (or ``intraday_return`` = (close − open)/open). The network fetch (:15-24) and the
entropy prints (:46-53) are out of scope. ``future_inputs`` restates ``generate_future_dates``
(:67-90). ``load_series`` reads many tickers at once into the ragged lists the batched engine
(``Engine`` / ``Scipy().minimize_stream`` / ``distributed.fit_assets``) consumes.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import pandas as pd
import torch

EOD_COLUMNS = ("date", "open", "high", "low", "close", "adjusted_close", "volume")


def _frame(csv_path: str, train_start_date: str) -> pd.DataFrame:
    df = pd.read_csv(csv_path)
    missing = [c for c in ("date", "open", "close") if c not in df.columns]
    if missing:
        raise ValueError(f"{csv_path}: not an EODHD end-of-day CSV (missing {missing})")
    df["date"] = pd.to_datetime(df["date"])
    df["day_of_year"] = (df["date"] - pd.Timestamp(train_start_date)).dt.days
    ret = df["close"].pct_change()
    df["return"] = ret.fillna(ret.iloc[1]) if len(df) > 1 else ret.fillna(0.0)
    df["intraday_return"] = (df["close"] - df["open"]) / df["open"]
    return df


def process_csv(csv_path: str, train_start_date: str, predict_Y: str = "return"):
    """(X [N,1], Y [N,1] float64 tensors, dates, mean, std) as DataHandler.process_data."""
    df = _frame(csv_path, train_start_date)
    col = df[predict_Y]
    mean, std = col.mean(), col.std()
    y = ((col - mean) / std).to_numpy(dtype=np.float64).reshape(-1, 1)
    x = df["day_of_year"].to_numpy(dtype=np.float64).reshape(-1, 1)
    return torch.from_numpy(x), torch.from_numpy(y), df["date"], float(mean), float(std)


def future_inputs(csv_path: str, train_start_date: str, period: str = "d", total_days: int = 90):
    """X_pred [H,1]: day offsets of the dates after the file's last date
    (daily: total_days days; weekly: total_days//7 week-ends; monthly: total_days//30 month-ends)."""
    last = pd.to_datetime(pd.read_csv(csv_path)["date"]).max()
    if period == "d":
        dates = pd.date_range(start=last + pd.Timedelta(days=1), periods=total_days, freq="D")
    elif period == "w":
        dates = pd.date_range(start=last + pd.DateOffset(weeks=1), periods=total_days // 7, freq="W")
    elif period == "m":
        dates = pd.date_range(start=last + pd.DateOffset(months=1), periods=total_days // 30, freq="ME")
    else:
        raise ValueError("Period must be 'd', 'w', or 'm'")
    x = (dates - pd.Timestamp(train_start_date)).days.to_numpy(dtype=np.float64)
    return torch.from_numpy(x.reshape(-1, 1))


def load_series(csv_paths: Sequence[str], train_start_date: str, predict_Y: str = "return"
                ) -> Tuple[List[Tuple[torch.Tensor, torch.Tensor]], List[Dict]]:
    """Many tickers → ([(X, Y)], [{mean, std, dates, path}]) for the batched fitters."""
    series, meta = [], []
    for p in csv_paths:
        X, Y, dates, mean, std = process_csv(p, train_start_date, predict_Y)
        series.append((X, Y))
        meta.append(dict(mean=mean, std=std, dates=dates, path=p))
    return series, meta
