"""Host-side OneCycleLR + Adam step constants, precomputed once for the whole run.

Mirrors the reference's optimizer/scheduler pair (src/train_fibinet.py:78,84-92):
``torch.optim.Adam(lr, weight_decay)`` driven by ``OneCycleLR(max_lr=10*lr, epochs*steps,
pct_start=0.3, div_factor=25, final_div_factor=1000)`` with torch's defaults
(anneal 'cos', cycle_momentum=True -> beta1 cycled between 0.95 and 0.85, two phases).

Optimizer step t (1-based) runs with the scheduler values of index t-1 and Adam's bias
corrections ``1 - beta1_t ** t`` / ``1 - beta2 ** t`` computed in double precision as torch
does; the kernel receives them rounded to float32 (the precision torch's fp32 tensor ops apply
them at).  The table is uploaded once; the device step counter indexes it, so the train step
needs no host round trip and can be captured in a hipGraph.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np


class OneCycle:
    def __init__(self, total_steps: int, base_lr: float = 1e-3, max_lr_mult: float = 10.0, pct_start: float = 0.3,
                 div_factor: float = 25.0, final_div_factor: float = 1000.0, max_momentum: float = 0.95,
                 base_momentum: float = 0.85):
        if total_steps <= 0:
            raise ValueError(f"Expected positive integer total_steps, but got {total_steps}")
        self.total_steps = total_steps
        self.max_lr = base_lr * max_lr_mult
        self.initial_lr = self.max_lr / div_factor
        self.min_lr = self.initial_lr / final_div_factor
        self.phases = [
            (float(pct_start * total_steps) - 1, self.initial_lr, self.max_lr, max_momentum, base_momentum),
            (total_steps - 1, self.max_lr, self.min_lr, base_momentum, max_momentum),
        ]

    @staticmethod
    def _cos(start: float, end: float, pct: float) -> float:
        return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)

    def at(self, step_num: int) -> Tuple[float, float]:
        """(lr, beta1) the scheduler holds after ``step_num`` scheduler steps."""
        if step_num > self.total_steps:
            raise ValueError(f"Tried to step {step_num} times. The specified number of total steps is "
                             f"{self.total_steps}")
        start = 0.0
        for i, (end, lr0, lr1, m0, m1) in enumerate(self.phases):
            if step_num <= end or i == len(self.phases) - 1:
                pct = (step_num - start) / (end - start)
                return self._cos(lr0, lr1, pct), self._cos(m0, m1, pct)
            start = end
        raise AssertionError("unreachable")


def adam_table(total_steps: int, base_lr: float = 1e-3, beta2: float = 0.999,
               sched: OneCycle = None, decoupled_wd: float = 0.0) -> Tuple[np.ndarray, List[float]]:
    """float32 [total_steps + 1, 8] rows (1 - beta1, -lr/bc1, sqrt(bc2), 1/sqrt(bc2), dmul, 0, 0, 0)
    for optimizer steps 1..T (column 4: the table-row step multiplies by it; dmul = 1 - lr * wd,
    torch.optim.AdamW's decoupled decay, when ``decoupled_wd`` is given, else 1), and the lr of
    each step.  The extra last row repeats step T (the device counter saturates there)."""
    sched = sched or OneCycle(total_steps, base_lr)
    tab = np.zeros((total_steps + 1, 8), dtype=np.float32)
    lrs = []
    for t in range(1, total_steps + 1):
        lr, b1 = sched.at(t - 1)
        step = float(t)
        bc1 = 1 - b1 ** step
        bc2 = 1 - beta2 ** step
        step_size = lr / bc1
        tab[t - 1, :5] = (1 - b1, -step_size, bc2 ** 0.5, 1.0 / bc2 ** 0.5, 1.0 - lr * decoupled_wd)
        lrs.append(lr)
    tab[total_steps] = tab[total_steps - 1]
    return tab, lrs
