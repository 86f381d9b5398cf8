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
    # psiref-tracking policies: the lane-reference interpolant (an object with grid ``g`` and
    # values ``v``, highway_branch_dyn.LinearInterpolant) the kernels evaluate psiref(X) from
    lane_ref: object = None

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


def lane_ref_of(policies):
    """The one lane reference the psiref policies of a policy list share, as (grid, values),
    or None when no policy tracks one."""
    refs = [p.lane_ref for p in policies if p.lane_ref is not None]
    if not refs:
        return None
    r0 = refs[0]
    for r in refs[1:]:
        if r is not r0 and not (len(r.g) == len(r0.g) and (r.g == r0.g).all() and (r.v == r0.v).all()):
            raise ValueError("the psiref policies of one model must track the same lane reference")
    return r0.g, r0.v


KIND_NAMES = {abi.POL_MAINTAIN: "maintain", abi.POL_BRAKE: "brake", abi.POL_LC: "lc",
              abi.POL_MAINTAIN_TRACKV: "maintain_trackV", abi.POL_FORWARD: "forward",
              abi.POL_STOP: "stop", abi.POL_MAINTAIN_PSIREF: "maintain(psiref)",
              abi.POL_MAINTAIN_TRACKV_PSIREF: "maintain_trackV(psiref)", abi.POL_BRAKE_PSIREF: "brake(psiref)"}
