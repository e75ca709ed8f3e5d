"""Probe-only stand-in for `hurry.filesize` (absent offline).

The reference only uses `size()` to pretty-print memories in log lines
(`core/utils/input_to_data.py:62-63,76,79`); the value never reaches the model.
Used exclusively by tools/gen_golden.py in the build container.
"""


def size(b):
    return f"{b}B"
