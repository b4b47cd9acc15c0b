"""The tuned-plan file format, pinned against the native writer on the CPU (a header added to
the plan files broke the GPU harness's parser and stopped the driver's GPU suite at test 32).  The plan API of
libstereo_amd.so needs no device: entries are seeded in-process, written by conv_plan_save
(csrc/runtime/runtime.cpp), then read back by the Python reader every test uses and by the native loader.
Also pins the loader's rejection rules: a file without a header or with another build's header is not
trusted, and an entry naming a tactic this build does not have is dropped instead of failing the launch."""
import pytest

from stereoalgorithms_amd import _native as N
from stereoalgorithms_amd.utils.plan import read_plan

pytestmark = pytest.mark.skipif(not N.available(), reason="native library not built")

KEYS = ["gfx950|1,120,160,384|128.256.|k1x3x3|s1,1,1|p0,1,1|d1,1|o120x160|D0,0|c256,3456|e1,0,0,0,0|w1",
        "gfx950|1,60,80,256|256.|k1x1x1|s1,1,1|p0,0,0|d1,1|o60x80|D0,0|c128,256|e0,0,0,0,0|w0"]


def _lib():
    lib = N.dev()
    lib.sa_conv_plan_clear()
    return lib


def test_native_writer_roundtrip(tmp_path):
    lib = _lib()
    lib.sa_conv_plan_put(KEYS[0].encode(), 26, 1, 41.5)
    lib.sa_conv_plan_put(KEYS[1].encode(), 3, 0, 7.25)
    lib.sa_conv_plan_put(b"gfx950|untuned", -1, 1, 1e30)  # no tactic found: never written
    path = tmp_path / "x.plan"
    assert lib.sa_conv_plan_save(str(path).encode(), "\n".join(KEYS + ["gfx950|untuned", KEYS[0]]).encode()) == 0
    build, entries = read_plan(path)
    assert build == lib.sa_plan_build_id().decode() and len(build) == 16
    assert [(e.key, e.cfg, e.splitk, e.us) for e in entries] == [(KEYS[0], 26, 1, 41.5), (KEYS[1], 3, 0, 7.25)]
    # the native loader reads its own file back
    lib.sa_conv_plan_clear()
    assert lib.sa_conv_plan_load(str(path).encode()) == 2
    assert lib.sa_conv_plan_entries() == 2


def test_loader_rejects_stale_and_headerless_files(tmp_path):
    lib = _lib()
    body = f"{KEYS[0]} 26 1 41.5\n"
    stale = tmp_path / "stale.plan"
    stale.write_text("# sa-plan build=0000000000000000\n" + body)
    assert lib.sa_conv_plan_load(str(stale).encode()) == -2
    legacy = tmp_path / "legacy.plan"  # a plan written before headers existed
    legacy.write_text(body)
    assert lib.sa_conv_plan_load(str(legacy).encode()) == -2
    assert lib.sa_conv_plan_load(str(tmp_path / "absent.plan").encode()) == -1
    assert lib.sa_conv_plan_entries() == 0


def test_loader_drops_unknown_tactics(tmp_path):
    lib = _lib()
    build = lib.sa_plan_build_id().decode()
    p = tmp_path / "edited.plan"
    p.write_text(f"# sa-plan build={build}\n{KEYS[0]} 9 1 10.0\n# comment\n{KEYS[1]} 3 1 5.0\n")
    assert lib.sa_conv_plan_load(str(p).encode()) == 1  # retired tactic 9 dropped, tactic 3 kept
    _, entries = read_plan(p)
    assert len(entries) == 2  # the reader itself is format-only


def test_tile_lds_footprints():
    """The per-tile-config LDS footprints the tuner's side-branch tie-break compares (SA_TUNE_LDS_TOL): every
    one-workgroup-per-CU DMA-ring / halo tile needs more than half the CU's 160 KB, the small register-staged and
    4-wave ring tiles leave room for other workgroups, the special-purpose kernels are not compared (-1)."""
    lib = N.dev()
    lds = {c: lib.sa_conv2d_tile_lds(c) for c in (0, 1, 3, 4, 5, 7, 14, 16, 26, 28, 22, 23, 24, 25, 99)}
    for c in (4, 26, 28):
        assert 81920 < lds[c] <= 163840, (c, lds[c])
    for c in (3, 5):
        assert 0 < lds[c] <= 81920, (c, lds[c])
    assert lds[3] < lds[0] and lds[5] < lds[4] and lds[16] <= 163840
    assert all(lds[c] == -1 for c in (22, 23, 24, 25, 99))


def test_plan_cache_append_switches_files(tmp_path, monkeypatch):
    """the SA_PLAN_CACHE appender verified the header once per PROCESS, so after switching to a
    second cache file (one per test case) entries were appended without a header and every later load rejected the
    file (-2).  The check is now keyed by path and repeated when the file was deleted."""
    lib = _lib()
    a, b = tmp_path / "a.plan", tmp_path / "b.plan"
    monkeypatch.setenv("SA_PLAN_CACHE", str(a))
    lib.sa_conv_plan_cache_append(KEYS[0].encode(), 26, 1, 41.5)
    monkeypatch.setenv("SA_PLAN_CACHE", str(b))
    lib.sa_conv_plan_cache_append(KEYS[1].encode(), 3, 0, 7.25)
    lib.sa_conv_plan_cache_append(KEYS[0].encode(), 28, 1, 40.0)
    build = lib.sa_plan_build_id().decode()
    for f, n in ((a, 1), (b, 2)):
        hdr, entries = read_plan(f)
        assert hdr == build and len(entries) == n, (f, hdr, entries)
        lib.sa_conv_plan_clear()
        assert lib.sa_conv_plan_load(str(f).encode()) == n
    # back to the first file after it was deleted: the header is written again
    a.unlink()
    monkeypatch.setenv("SA_PLAN_CACHE", str(a))
    lib.sa_conv_plan_cache_append(KEYS[1].encode(), 3, 1, 6.0)
    assert read_plan(a)[0] == build and lib.sa_conv_plan_load(str(a).encode()) == 1


def test_plan_load_counts_file_entries_not_new_ones(tmp_path):
    """loading a plan whose entries the process already holds (the second engine of the same
    shapes) reports the file's entry count, so 'loaded 0' only ever means an empty file."""
    lib = _lib()
    lib.sa_conv_plan_put(KEYS[0].encode(), 26, 1, 41.5)
    lib.sa_conv_plan_put(KEYS[1].encode(), 3, 0, 7.25)
    p = tmp_path / "x.plan"
    assert lib.sa_conv_plan_save(str(p).encode(), "\n".join(KEYS).encode()) == 0
    assert lib.sa_conv_plan_load(str(p).encode()) == 2  # nothing new, still 2
    empty = tmp_path / "empty.plan"
    empty.write_text(f"# sa-plan build={lib.sa_plan_build_id().decode()}\n")
    assert lib.sa_conv_plan_load(str(empty).encode()) == 0
    from stereoalgorithms_amd.utils.plan import plan_state, tactic_digest
    assert [plan_state(v) for v in (-3, -2, -1, 0, 5)] == ["not-consulted", "foreign-build", "absent", "empty", "loaded"]
    d1 = tactic_digest(p)
    q = tmp_path / "y.plan"  # same choices, other timings: same digest; another choice: different digest
    q.write_text(p.read_text().replace("41.5", "39"))
    assert tactic_digest(q) == d1
    q.write_text(p.read_text().replace(" 26 1 ", " 28 1 "))
    assert tactic_digest(q) != d1 and tactic_digest(tmp_path / "none.plan") is None


def test_pinned_table_survives_stale_local_plan(tmp_path):
    """a DP rank that merged rank 0's broadcast table pins it, so the plan file its engine loads at init (a
    stale file from an earlier job on that node) cannot override the broadcast choices; unpinned loads still merge."""
    lib = _lib()
    build = lib.sa_plan_build_id().decode()
    local = tmp_path / "local.plan"
    local.write_text(f"# sa-plan build={build}\n{KEYS[0]} 3 0 9.0\n{KEYS[1]} 4 0 8.0\n")
    lib.sa_conv_plan_put(KEYS[0].encode(), 26, 1, 41.5)  # the broadcast entry
    lib.sa_conv_plan_pin(1)
    try:
        assert lib.sa_conv_plan_load(str(local).encode()) == 2
    finally:
        lib.sa_conv_plan_pin(0)
    out = tmp_path / "out.plan"
    assert lib.sa_conv_plan_save(str(out).encode(), "\n".join(KEYS).encode()) == 0
    got = {e.key: (e.cfg, e.splitk) for e in read_plan(out)[1]}
    assert got == {KEYS[0]: (26, 1), KEYS[1]: (4, 0)}  # kept the pinned entry, added the missing one
    assert lib.sa_conv_plan_load(str(local).encode()) == 2  # unpinned: the file wins again
    assert lib.sa_conv_plan_save(str(out).encode(), "\n".join(KEYS).encode()) == 0
    assert {e.key: e.cfg for e in read_plan(out)[1]}[KEYS[0]] == 3
