"""gpflow.utilities.set_trainable / print_summary counterparts
(GPR/model_trainer.py:2,17; GPR/main.py:40-44)."""
from __future__ import annotations

import numpy as np

from .parameter import ArrayParameter, Parameter


def set_trainable(obj, flag: bool) -> None:
    """Set ``trainable`` on a Parameter or on every Parameter of a kernel/likelihood/model."""
    if isinstance(obj, (Parameter, ArrayParameter)):
        obj.trainable = bool(flag)
        return
    params = getattr(obj, "parameters", None)
    if params is None:
        raise TypeError(f"cannot set_trainable on {type(obj).__name__}")
    for p in params:
        p.trainable = bool(flag)


def summary_rows(model):
    rows = []
    paths = model._param_paths() if hasattr(model, "_param_paths") else [
        (n, p) for n, p in model._param_paths("")]
    for name, p in paths:
        if isinstance(p, ArrayParameter):
            v = p.value
            rows.append((name, "Parameter", p.transform_name, p.trainable, str(tuple(v.shape)), "float64",
                         np.array2string(v.ravel()[:3], precision=4) + ("..." if v.size > 3 else "")))
        else:
            rows.append((name, "Parameter", p.transform_name, p.trainable, "()", "float64", p.value))
    return rows


def print_summary(model, fmt: str = None) -> None:
    rows = summary_rows(model)
    hdr = ("name", "class", "transform", "trainable", "shape", "dtype", "value")
    cells = [hdr] + [tuple(str(c) if not isinstance(c, float) else f"{c:.8g}" for c in r) for r in rows]
    widths = [max(len(r[i]) for r in cells) for i in range(len(hdr))]
    line = "+" + "+".join("-" * (w + 2) for w in widths) + "+"
    print(line)
    for k, r in enumerate(cells):
        print("| " + " | ".join(c.ljust(w) for c, w in zip(r, widths)) + " |")
        if k == 0:
            print(line.replace("-", "="))
    print(line)
