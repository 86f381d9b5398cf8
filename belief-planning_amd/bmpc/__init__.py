"""Internal package of the MI355X branch-MPC drop-in (ctypes boundary, plans, tracing)."""
