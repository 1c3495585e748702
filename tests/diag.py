"""Diagnostics shared by the tests that run the framework in subprocesses."""


def failure_text(err: str) -> str:
    """A failed run's stderr for the assertion message: the native backtrace
    of a fatal signal in full (the crash handler's frames, which name the
    library and offset that called free() — the Python tail alone cut them
    off), then the tail."""
    mark = "heat2d: fatal signal, native backtrace:"
    i = err.find(mark)
    head = err[max(0, i - 600):i + 6000] + "\n...\n" if i >= 0 else ""
    return head + err[-3000:]
