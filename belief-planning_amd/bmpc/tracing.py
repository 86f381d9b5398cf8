"""Policy tracer: lowers the reference's backup-policy lambdas to kernel descriptors.

The reference builds its CasADi graphs by calling each policy lambda with a symbolic
``SX`` vector; the policy helpers dispatch on ``isinstance(x, casadi.SX)``
(``highway_branch_dyn.py:54-148``, ``quadruped_branch_dyn.py:34-54``).  Here the same
lambdas are called with a :class:`Tracer`; the helpers in ``highway_branch_dyn`` /
``quadruped_branch_dyn`` recognise it and return a :class:`PolicySpec` -- the descriptor
``(kind, params)`` that the GPU kernels evaluate in closed form.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import abi


class Tracer:
    """Stand-in for the symbolic state vector; indexing it is an error (a policy that the
    tracer does not understand must not be silently mis-lowered)."""

    def __getitem__(self, item):
        raise TypeError("policy lambda indexed the traced state directly; only the library's "
                        "backup_* helpers can be lowered to GPU policy descriptors")


@dataclass(frozen=True)
class PolicySpec:
    kind: int
    params: tuple = ()

    def as_row(self):
        return (self.kind, self.params)


def trace(policies):
    """Call each backup lambda with a Tracer and collect the descriptors."""
    out = []
    for f in policies:
        spec = f(Tracer())
        if not isinstance(spec, PolicySpec):
            raise TypeError(f"backup policy {f!r} did not lower to a PolicySpec (got {type(spec)})")
        out.append(spec)
    return out


KIND_NAMES = {abi.POL_MAINTAIN: "maintain", abi.POL_BRAKE: "brake", abi.POL_LC: "lc",
              abi.POL_MAINTAIN_TRACKV: "maintain_trackV", abi.POL_FORWARD: "forward",
              abi.POL_STOP: "stop"}
