"""Native builds are keyed by source CONTENT, not mtime (the .so files travel to the GPU box
untracked, with fresh mtimes): a touched-but-identical source does not rebuild, a changed
one does (cs230_distributed_machine_learning_amd/build.py)."""
import os
import time

from cs230_distributed_machine_learning_amd import build as b


def _mini_tree(tmp_path, body):
    csrc = tmp_path / "csrc"
    (csrc / "runtime").mkdir(parents=True)
    (csrc / "kernels").mkdir()
    src = csrc / "runtime" / "a.cpp"
    src.write_text(body)
    return csrc, src


def test_cpu_lib_rebuilds_on_content_change_only(tmp_path, monkeypatch):
    csrc, src = _mini_tree(tmp_path, 'extern "C" int dml_probe() { return 1; }\n')
    lib = tmp_path / "lib"
    monkeypatch.setattr(b, "CSRC", str(csrc))
    monkeypatch.setattr(b, "LIB", str(lib))
    monkeypatch.setattr(b, "CPU_LIB", str(lib / "libdml_cpu.so"))
    out = b.build_cpu()
    m0 = os.path.getmtime(out)
    time.sleep(1.1)
    os.utime(src)                          # newer mtime, same bytes
    assert b.build_cpu() == out and os.path.getmtime(out) == m0
    src.write_text('extern "C" int dml_probe() { return 2; }\n')
    b.build_cpu()
    assert os.path.getmtime(out) > m0      # changed content rebuilt


def test_stale_by_hash_covers_flags(tmp_path):
    src = tmp_path / "x.cpp"
    src.write_text("int x;\n")
    tgt = tmp_path / "x.o"
    tgt.write_text("obj")
    assert b._stale_by_hash(str(tgt), [str(src)], ["-O3"])          # no stamp yet
    b._stamp(str(tgt), [str(src)], ["-O3"])
    assert not b._stale_by_hash(str(tgt), [str(src)], ["-O3"])
    assert b._stale_by_hash(str(tgt), [str(src)], ["-O2"])          # different flags


def test_hash_is_path_independent_and_builds_are_locked(tmp_path, monkeypatch):
    """A tree moved to another directory (the GPU box's scratch copy) keeps its stamps
    valid, and the build writes through a per-process temporary under a file lock (ranks
    that start together never load a half-written library)."""
    import shutil
    import threading

    csrc, src = _mini_tree(tmp_path / "a", 'extern "C" int dml_probe() { return 1; }\n')
    monkeypatch.setattr(b, "CSRC", str(csrc))
    h0 = b._src_hash([str(src)], ["-I", str(csrc / "kernels"), "-O3"])
    moved = tmp_path / "b"
    shutil.copytree(tmp_path / "a", moved)
    monkeypatch.setattr(b, "CSRC", str(moved / "csrc"))
    h1 = b._src_hash([str(moved / "csrc" / "runtime" / "a.cpp")], ["-I", str(moved / "csrc" / "kernels"), "-O3"])
    assert h0 == h1
    lib = tmp_path / "lib"
    monkeypatch.setattr(b, "LIB", str(lib))
    monkeypatch.setattr(b, "CPU_LIB", str(lib / "libdml_cpu.so"))
    errs = []

    def one():
        try:
            b.build_cpu()
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=one) for _ in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs and os.path.exists(lib / "libdml_cpu.so")
    assert not [p for p in os.listdir(lib) if p.endswith(".tmp")]
