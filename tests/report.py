"""Per-config parity lines collected during a run and printed by
conftest.pytest_terminal_summary (the tail of ``pytest -q`` is evidence)."""

LINES = []


def record(line):
    LINES.append(line)
    print(line, flush=True)
