"""Reader for the tuned-plan files the native engine writes (csrc/runtime/runtime.cpp conv_plan_save / the
SA_PLAN_CACHE appender): a ``# sa-plan build=<id>`` header, then one ``<key> <cfg> <splitk> <us>`` line per conv
shape.  The key itself has no spaces.  Lines starting with ``#`` are comments.  Tests and tools parse plans through
this one function so a format change breaks one place (tests/test_plan_format_cpu.py pins it against the native
writer)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class PlanEntry:
    key: str
    cfg: int
    splitk: int
    us: float


def read_plan(path) -> tuple[str | None, list[PlanEntry]]:
    """Returns (build id from the header or None, entries in file order)."""
    build = None
    entries: list[PlanEntry] = []
    with open(path) as f:
        for i, line in enumerate(f):
            line = line.strip()
            if not line:
                continue
            if line.startswith("#"):
                if build is None and "build=" in line:
                    build = line.split("build=", 1)[1].split()[0]
                continue
            key, cfg, sk, us = line.rsplit(" ", 3)
            entries.append(PlanEntry(key, int(cfg), int(sk), float(us)))
    return build, entries


def tactic_digest(path) -> str | None:
    """16-hex digest of a plan's tactic CHOICES: the sorted (key, cfg, splitk) triples plus the build id (timings
    excluded).  Two processes -- or two ranks of a DP job -- with equal digests launch identical kernels for every
    conv shape.  None when the file does not exist."""
    import hashlib
    import os
    if not path or not os.path.exists(path):
        return None
    build, entries = read_plan(path)
    h = hashlib.sha256((build or "").encode())
    for e in sorted(entries, key=lambda e: e.key):
        h.update(f"\n{e.key} {e.cfg} {e.splitk}".encode())
    return h.hexdigest()[:16]


PLAN_STATES = {-3: "not-consulted", -2: "foreign-build", -1: "absent"}


def plan_state(loaded: int) -> str:
    """The engine's plan-file outcome at build (sa_engine_plan_status 'loaded'): 'absent' (no file, every shape
    tuned), 'foreign-build' (written by another library build, ignored), 'empty' (file found, no entries),
    'loaded' (file found with entries), 'not-consulted' (tuning disabled)."""
    if loaded in PLAN_STATES:
        return PLAN_STATES[loaded]
    return "empty" if loaded == 0 else "loaded"
