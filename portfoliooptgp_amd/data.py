"""On-disk input format → device-ready series.

The reference reads EODHD end-of-day CSVs (``date,open,high,low,close,adjusted_close,volume``,
e.g. ``Stocks/AAPL_EOD/AAPL_us_d.csv``) and turns each into a GP training set in
``GPR/data_handler.py:26-65``: X = days since ``train_start_date`` (unnormalised), Y = the
z-scored (pandas ddof=1) ``return`` = ``close.pct_change()`` with row 0 filled by row 1's
return (or ``intraday_return`` = (close − open)/open). The network fetch (:15-24) and the
entropy prints (:46-53) are out of scope. ``future_inputs`` restates ``generate_future_dates``
(:67-90). ``load_series`` reads many tickers at once into the ragged lists the batched engine
(``Engine`` / ``Scipy().minimize_stream`` / ``distributed.fit_assets``) consumes;
``load_batch`` does the same with the files parsed on a thread pool and every series landing on
the device through ONE pinned host block and ONE host-to-device copy.

The index series (``Stocks/Index/*/<name>.csv``) come from investing.com
(``"Date","Price","Open","High","Low","Vol.","Change %"``, newest first, ``MM/DD/YYYY``);
``convert_investing_csv`` restates ``handle.py:38-75`` (``convert_csv`` + ``sort_csv``) that turns
them into the ``date,open,high,low,close,change,volume`` files next to them
(``<name>_us_d.csv``), byte for byte (tests/test_data.py against the reference's own pairs).
"""
from __future__ import annotations

import csv
import io
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import pandas as pd
import torch

EOD_COLUMNS = ("date", "open", "high", "low", "close", "adjusted_close", "volume")
INVESTING_OUT_COLUMNS = ("date", "open", "high", "low", "close", "change", "volume")


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


def investing_rows(input_file: str) -> List[Dict[str, str]]:
    """The rows of an investing.com export in the converted schema, oldest first
    (``handle.py:38-59`` per row: date ``MM/DD/YYYY`` -> ``YYYY-MM-DD``, ``Price`` -> close, an
    empty ``Vol.`` -> ``'0'``; values kept as the file's strings, e.g. ``40,792.79``; then
    ``sort_csv``'s stable sort by date, ``handle.py:61-75``)."""
    rows = []
    with open(input_file, "r", newline="") as f:
        reader = csv.reader(f)
        next(reader)  # header (the file's BOM is part of it)
        for row in reader:
            date = datetime.strptime(row[0].strip('"'), "%m/%d/%Y").strftime("%Y-%m-%d")
            rows.append({"date": date, "open": row[2].strip('"'), "high": row[3].strip('"'),
                         "low": row[4].strip('"'), "close": row[1].strip('"'), "change": row[6].strip('"'),
                         "volume": row[5].strip('"') if row[5].strip('"') else "0"})
    rows.sort(key=lambda r: datetime.strptime(r["date"], "%Y-%m-%d"))
    return rows


def convert_investing_csv(input_file: str, output_file: Optional[str] = None) -> str:
    """Convert an investing.com export to the ``date,open,high,low,close,change,volume`` CSV the
    reference keeps beside it; returns the text (csv module defaults: ``\\r\\n`` line ends, fields
    with commas quoted) and writes it to ``output_file`` when given."""
    buf = io.StringIO(newline="")
    w = csv.DictWriter(buf, fieldnames=list(INVESTING_OUT_COLUMNS))
    w.writeheader()
    w.writerows(investing_rows(input_file))
    text = buf.getvalue()
    if output_file is not None:
        with open(output_file, "w", newline="") as f:
            f.write(text)
    return text


def load_batch(csv_paths: Sequence[str], train_start_date: str, predict_Y: str = "return",
               device=None, workers: int = 8):
    """Many tickers -> device-resident series for the batched fitters.

    The files are parsed concurrently (pandas' C parser releases the GIL), each series'
    (X, Y) written into one pinned [2, Σ N_b] float64 host block, which goes to ``device`` in one
    copy; the returned X_b / Y_b ([N_b, 1]) are views of that device block (``Engine`` and
    ``GPR`` take them as they are). Returns ([(X_b, Y_b)], [{mean, std, dates, path, n}]) with the
    values of ``process_csv`` bit for bit."""
    paths = list(csv_paths)
    with ThreadPoolExecutor(max_workers=max(1, min(workers, len(paths) or 1))) as ex:
        parts = list(ex.map(lambda p: process_csv(p, train_start_date, predict_Y), paths))
    sizes = [int(X.shape[0]) for X, *_ in parts]
    total = sum(sizes)
    pin = device is not None and torch.device(device).type == "cuda"
    host = torch.empty((2, total), dtype=torch.float64, pin_memory=pin)
    off = 0
    for (X, Y, *_), nb in zip(parts, sizes):
        host[0, off:off + nb] = X[:, 0]
        host[1, off:off + nb] = Y[:, 0]
        off += nb
    dev = host.to(device, non_blocking=pin) if device is not None else host
    series, meta, off = [], [], 0
    for p, (_, _, dates, mean, std), nb in zip(paths, parts, sizes):
        series.append((dev[0, off:off + nb].view(nb, 1), dev[1, off:off + nb].view(nb, 1)))
        meta.append(dict(mean=mean, std=std, dates=dates, path=p, n=nb))
        off += nb
    if pin:  # read-only inputs: their band-table boxes are computed once (engine.mark_immutable)
        from .engine import mark_immutable
        mark_immutable(*(t for xy in series for t in xy))
    return series, meta
