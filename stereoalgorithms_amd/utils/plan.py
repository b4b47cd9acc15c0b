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
