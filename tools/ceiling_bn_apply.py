"""Ceiling of folding the BN1 backward apply into its consumers: the driver's
graph-replayed cfg3 step (bench.py) with the apply of every fused
BN1 / PReLU backward (ops.bn_backward_rows -> rr_bn_bwd_apply, the 11
bn_bwd_apply8 launches of a step at the HBM wall) skipped -- the PReLU-masked
gradient gm goes to conv1's dgrad and weight grad as if it were dt1.  Timing
only: the results are WRONG in the skipped mode.  Nothing in the library or
the package is switched: the skip is a monkeypatch of this process.

    python tools/ceiling_bn_apply.py [ROUNDS]

alternates `base` and `skip` child processes ROUNDS times (default 3) and
prints one line per run plus the medians."""
import json
import os
import statistics
import subprocess
import sys

R_ = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def child(mode):
    sys.path.insert(0, R_)
    sys.path.insert(0, os.path.join(R_, "image-restoration-for-road-sign-recognition-in-autonomous-driving_amd"))
    from roadrestore import engine, ops
    if mode == "skip":
        import ctypes as C
        import torch

        def no_apply(gm, part, rows, arows, t0, mean0, inv0, gamma0, outs=None, eval_mode=False,
                     dbias=None):
            # ops.bn_backward_rows without its rr_bn_bwd_apply launch
            Cc = gm.shape[-1]
            P = gm.numel() // Cc
            dev = gm.device
            d = ops.BnBwdDesc(ops.rr_dtype(gm.dtype), P, Cc, 0, 1)
            ops._set_eval(d, eval_mode, dbias)
            o = outs or {}
            dg0 = o.get("dgamma0")
            dg0 = torch.empty(Cc, dtype=torch.float32, device=dev) if dg0 is None else dg0
            db0 = o.get("dbeta0")
            db0 = torch.empty_like(dg0) if db0 is None else db0
            dal = o.get("dalpha")
            dal = torch.empty(1, dtype=torch.float32, device=dev) if dal is None else dal
            coef = torch.empty(Cc * 6, dtype=torch.float32, device=dev)
            L = ops.lib()
            ws = ops._ws(L.rr_bn_bwd_finalize_rows_workspace(Cc, rows), dev)
            apart = part[rows * Cc * 3:]
            p = ops._p
            L.check(L.rr_bn_bwd_finalize_rows(C.byref(d), rows, p(part), arows, p(apart), p(gamma0),
                                              p(inv0), p(dg0), p(db0), p(dal), p(coef), p(ws),
                                              ws.numel(), ops.stream()), "rr_bn_bwd_finalize_rows")
            return dict(dt0=gm, dgamma0=dg0, dbeta0=db0, dalpha=dal)
        engine.ops.bn_backward_rows = no_apply
    import bench
    sys.argv = ["bench.py", "--no-cpu-baseline", "--no-probe", "--steps", "30"]
    bench.main()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    res = {"base": [], "skip": []}
    for _ in range(rounds):
        for mode in ("base", "skip"):
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode],
                                 capture_output=True, text=True, timeout=300)
            if out.returncode:
                print(out.stderr[-2000:], file=sys.stderr)
                raise SystemExit(out.returncode)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[mode].append(d["ms_per_step"])
            print(mode, d["value"], d["ms_per_step"], flush=True)
    mb, ms = statistics.median(res["base"]), statistics.median(res["skip"])
    print(json.dumps({"base_ms": mb, "skip_bn1_apply_ms": ms, "ceiling_frac": round((mb - ms) / mb, 4),
                      "runs": res}))


if __name__ == "__main__":
    main()
