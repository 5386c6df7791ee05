"""RR_PATH (csrc/common.h rr_path, roadrestore._lib.path_flag): the one
kernel-path override the parity tests use to check one shipped kernel
against another on the same shape."""
import os


def set_path(monkeypatch, key, value):
    """Set ``key=value`` in RR_PATH for this test, keeping the other keys."""
    cur = {}
    for item in os.environ.get("RR_PATH", "").split(","):
        k, sep, v = item.partition("=")
        if sep:
            cur[k] = v
    cur[key] = str(value)
    monkeypatch.setenv("RR_PATH", ",".join(f"{k}={v}" for k, v in cur.items()))
