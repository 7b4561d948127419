"""Persistent kernel-selection database (ops/tunedb.py): round trip, merge of concurrent writers,
pruning of stale library sections, and the backend's use of it (a database hit is never re-timed)."""
import json

from distributed_resnet_tensorflow_amd.ops.tunedb import TuneDB


def test_round_trip_and_merge(tmp_path):
    p = tmp_path / "db.json"
    a = TuneDB("gfx950/256cu|aaaa", p)
    a.put_conv((128, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, 1, True, 0, False, False, True, False), (25, -512))
    a.put_wgrad((128, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, True, False), (512, 7, True, 8))
    assert a.save() and not a.dirty
    assert not a.save()                      # nothing new: no write
    b = TuneDB("gfx950/256cu|aaaa", p)       # a second process of the same library
    assert b.get_conv((128, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, 1, True, 0, False, False, True, False)) == (25, -512)
    assert b.get_wgrad((128, 56, 56, 64, 64, 3, 3, 56, 56, 1, 1, 1, True, False)) == (512, 7, True, 8)
    assert b.get_conv((1, 2, 3)) is None
    b.put_conv((1, 2, 3), (0, 1))
    a.put_conv((4, 5, 6), (3, 2))            # concurrent writer: both keys survive
    b.save()
    a.save()
    c = TuneDB("gfx950/256cu|aaaa", p)
    assert c.get_conv((1, 2, 3)) == (0, 1) and c.get_conv((4, 5, 6)) == (3, 2)


def test_stale_library_sections_are_dropped(tmp_path):
    p = tmp_path / "db.json"
    old = TuneDB("gfx950/256cu|old0", p)
    old.put_conv((1,), (1, 1))
    old.save()
    other_dev = TuneDB("gfx942/304cu|old0", p)
    other_dev.put_conv((1,), (2, 1))
    other_dev.save()
    new = TuneDB("gfx950/256cu|new0", p)
    assert new.get_conv((1,)) is None         # another library build: never reused
    new.put_conv((1,), (5, 1))
    new.save()
    secs = json.loads(p.read_text())["sections"]
    assert set(secs) == {"gfx950/256cu|new0", "gfx942/304cu|old0"}


def test_version_mismatch_and_corrupt_file_are_ignored(tmp_path):
    p = tmp_path / "db.json"
    p.write_text(json.dumps({"version": 999, "sections": {"s|h": {"conv": {"1": [7, 1]}}}}))
    assert TuneDB("s|h", p).get_conv((1,)) is None
    p.write_text("{not json")
    db = TuneDB("s|h", p)
    assert db.get_conv((1,)) is None
    db.put_conv((1,), (3, 1))
    assert db.save() and TuneDB("s|h", p).get_conv((1,)) == (3, 1)


def test_disabled_by_env(tmp_path, monkeypatch):
    monkeypatch.setenv("DRN_TUNE_DB", "off")
    db = TuneDB("s|h")
    db.put_conv((1,), (3, 1))
    assert db.path is None and not db.save()


def test_section_hash_covers_only_tuning_sources(tmp_path):
    """The database section hash (build.tune_hash) follows the conv / weight-gradient / stem
    kernels and the shared headers; editing another kernel changes the library hash only."""
    from distributed_resnet_tensorflow_amd.ops import build
    k, inc = tmp_path / "kernels", tmp_path / "include"
    k.mkdir()
    inc.mkdir()
    for n in build.TUNE_SOURCES + ("pool.hip", "sgd.hip"):
        (k / n).write_text(f"// {n}\n")
    (inc / "drn_conv.h").write_text("// header\n")
    t0, s0 = build.tune_hash(k, inc), build.source_hash(k, inc)
    (k / "pool.hip").write_text("// pool, edited\n")
    assert build.tune_hash(k, inc) == t0 and build.source_hash(k, inc) != s0
    (k / "conv_wgrad.hip").write_text("// wgrad, edited\n")
    assert build.tune_hash(k, inc) != t0
    t1 = build.tune_hash(k, inc)
    (inc / "drn_conv.h").write_text("// header, edited\n")
    assert build.tune_hash(k, inc) != t1


def test_shipped_database_matches_the_tree():
    """The shipped database's section is keyed by the current tuning-source hash, so a bench run
    on an MI355X uses it instead of re-tuning."""
    from distributed_resnet_tensorflow_amd.ops import build
    from distributed_resnet_tensorflow_amd.ops.tunedb import SYSTEM_PATH
    secs = json.loads(SYSTEM_PATH.read_text())["sections"]
    assert any(s.endswith("|" + build.tune_hash()[:16]) for s in secs), list(secs)


def test_system_database_is_read_only_and_read_first(tmp_path, monkeypatch):
    """The shipped (system) database is consulted before the user database and never written:
    a run's own quick tunings land in the user file only (a test run must not
    replace the shipped MI355X choices)."""
    sysdb, user = tmp_path / "system.json", tmp_path / "user.json"
    s = TuneDB("gfx950/256cu|abcd", sysdb)
    s.put_conv((1, 2), (7, 1))
    s.put_wgrad((3,), (512, 2, False, 8))
    assert s.save()
    before = sysdb.read_text()
    u = TuneDB("gfx950/256cu|abcd", user, system=sysdb)
    assert u.get_conv((1, 2)) == (7, 1) and u.get_wgrad((3,)) == (512, 2, False, 8)
    u.put_conv((1, 2), (9, 1))              # a quick re-tune of a shipped geometry...
    u.put_conv((5, 6), (4, 1))
    assert u.save()
    assert sysdb.read_text() == before      # ...never touches the system file
    again = TuneDB("gfx950/256cu|abcd", user, system=sysdb)
    assert again.get_conv((1, 2)) == (7, 1)  # the system choice wins
    assert again.get_conv((5, 6)) == (4, 1)  # the user file fills the gaps
    monkeypatch.setenv("DRN_TUNE_DB", str(sysdb))
    from distributed_resnet_tensorflow_amd.ops import tunedb
    monkeypatch.setattr(tunedb, "SYSTEM_PATH", sysdb)
    w = TuneDB("gfx950/256cu|abcd")         # pointed at the system file: writes are refused
    w.put_conv((8,), (1, 1))
    assert not w.save() and sysdb.read_text() == before


def test_system_database_can_be_switched_off(tmp_path, monkeypatch):
    """DRN_TUNE_DB_SYSTEM=off (scripts/make_tune_db.py, gpu_make_db.sh): a rebuild re-times every
    geometry instead of taking the shipped choices, so its output is a complete section."""
    from distributed_resnet_tensorflow_amd.ops import tunedb
    sysdb, user = tmp_path / "system.json", tmp_path / "user.json"
    s = TuneDB("gfx950/256cu|abcd", sysdb)
    s.put_conv((1, 2), (7, 1))
    assert s.save()
    monkeypatch.setattr(tunedb, "SYSTEM_PATH", sysdb)
    monkeypatch.setenv("DRN_TUNE_DB", str(user))
    assert TuneDB("gfx950/256cu|abcd").get_conv((1, 2)) == (7, 1)
    monkeypatch.setenv("DRN_TUNE_DB_SYSTEM", "off")
    db = TuneDB("gfx950/256cu|abcd")
    assert db.get_conv((1, 2)) is None
    db.put_conv((1, 2), (3, 1))
    assert db.save() and json.loads(user.read_text())["sections"]["gfx950/256cu|abcd"]["conv"]["1,2"] == [3, 1]
