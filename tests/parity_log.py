"""Achieved parity errors of the GPU tests (max |device - reference|, and the reference's scale),
collected per quantity so that a run reports how far inside its tier each test landed."""
import json
import os

RECORDS = []


def record(test, quantity, err, scale, tol):
    RECORDS.append({"test": test, "quantity": quantity, "err": float(err), "scale": float(scale),
                    "rel": float(err) / float(scale) if scale else None, "tol": float(tol)})


def dump(outdir):
    if not RECORDS or not os.path.isdir(outdir):
        return
    with open(os.path.join(outdir, f"parity_errors_{os.getpid()}.json"), "w") as fh:
        json.dump(RECORDS, fh, indent=0)
