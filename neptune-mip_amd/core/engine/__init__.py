"""MI355X engine: the C-ABI LP library binding (lp.py)."""
