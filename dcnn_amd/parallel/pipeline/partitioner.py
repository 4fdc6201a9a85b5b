"""Layer-range partitioners for pipeline stages.

* ``NaivePartitioner`` — equal *count* of top-level layers, the first ``rem`` stages take one
  extra (reference include/partitioner/naive_partitioner.hpp:13-32).
* ``FlopPartitioner`` — balances forward+backward FLOPs per stage (the reference's
  ``balance_load`` is a stub, include/pipeline/coordinator.hpp:331): contiguous partition of
  the per-layer cost vector minimising the maximum stage cost (exact DP, O(L^2 S)).
* ``CostPartitioner`` — same optimiser over any measured per-layer cost (e.g. the
  per-layer device times collected by ``Sequential`` profiling / stage load reports).
"""
from __future__ import annotations

from typing import List, Sequence

from ...nn.sequential import Partition, Sequential


class Partitioner:
    def get_partitions(self, model: Sequential, num_stages: int, input_shape=None) -> List[Partition]:
        raise NotImplementedError


class NaivePartitioner(Partitioner):
    def get_partitions(self, model, num_stages, input_shape=None):
        L = len(model.layers) if hasattr(model, "layers") else len(model)
        if num_stages <= 0 or num_stages > L:
            raise ValueError(f"cannot split {L} layers into {num_stages} stages")
        base, rem = divmod(L, num_stages)
        out, s = [], 0
        for i in range(num_stages):
            n = base + (1 if i < rem else 0)
            out.append(Partition(s, s + n))
            s += n
        return out


def balanced_split(costs: Sequence[float], num_stages: int) -> List[Partition]:
    """Contiguous split of ``costs`` into ``num_stages`` non-empty ranges minimising the max sum."""
    L = len(costs)
    if num_stages <= 0 or num_stages > L:
        raise ValueError(f"cannot split {L} layers into {num_stages} stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + float(c))
    INF = float("inf")
    # best[s][i]: minimal max-cost splitting first i layers into s stages
    best = [[INF] * (L + 1) for _ in range(num_stages + 1)]
    cut = [[0] * (L + 1) for _ in range(num_stages + 1)]
    best[0][0] = 0.0
    for s in range(1, num_stages + 1):
        for i in range(s, L - (num_stages - s) + 1):
            for j in range(s - 1, i):
                v = max(best[s - 1][j], pre[i] - pre[j])
                if v < best[s][i]:
                    best[s][i], cut[s][i] = v, j
    parts, i = [], L
    for s in range(num_stages, 0, -1):
        j = cut[s][i]
        parts.append(Partition(j, i))
        i = j
    return parts[::-1]


class FlopPartitioner(Partitioner):
    def __init__(self, input_shape=None):
        self.input_shape = input_shape

    def get_partitions(self, model, num_stages, input_shape=None):
        shape = list(input_shape or self.input_shape or [])
        if not shape:
            raise ValueError("FlopPartitioner needs the input shape [N, C, H, W]")
        f = model.forward_complexity(shape)
        b = model.backward_complexity(shape)
        return balanced_split([x + y for x, y in zip(f, b)], num_stages)


class CostPartitioner(Partitioner):
    def __init__(self, costs: Sequence[float]):
        self.costs = list(costs)

    def get_partitions(self, model, num_stages, input_shape=None):
        if len(self.costs) != len(model.layers):
            raise ValueError("one cost per top-level layer required")
        return balanced_split(self.costs, num_stages)


def create_partitioner(kind: str, input_shape=None) -> Partitioner:
    k = kind.lower()
    if k == "naive":
        return NaivePartitioner()
    if k in ("flops", "flop", "balanced"):
        return FlopPartitioner(input_shape)
    raise ValueError(f"unknown partitioner {kind}")
