"""The in-tree build's dependency list (CPU): every header the HIP sources include is a rebuild
trigger, so an edited header can never leave a stale libdrone2d_hip.so behind."""
from __future__ import annotations

import os
import re

import drone2d_amd  # noqa: F401
from drone2d_amd import _build


def _quoted_includes(path):
    out = []
    for line in open(path):
        m = re.match(r'\s*#\s*include\s+"([^"]+)"', line)
        if m:
            out.append(os.path.normpath(os.path.join(os.path.dirname(path), m.group(1))))
    return out


def test_every_included_header_is_a_dependency():
    deps = {os.path.normpath(p) for p in _build.env_headers()}
    todo, seen = [_build.SRC], set()
    while todo:
        f = todo.pop()
        if f in seen:
            continue
        seen.add(f)
        for inc in _quoted_includes(f):
            assert inc in deps, f"{inc} (included by {f}) is not in the build's dependency list"
            todo.append(inc)
    assert len(seen) >= 5  # d2d_hip.hip, d2d_kernels.h, d2d_device.h, d2d_curriculum.h, d2d_pmath.h, ...


def test_touching_any_header_triggers_rebuild(monkeypatch, tmp_path):
    out = str(tmp_path / "lib.so")
    open(out, "w").close()
    real = os.path.getmtime
    for hdr in _build.env_headers():
        def fake(p, hdr=hdr):
            p = os.path.normpath(p)
            if p == os.path.normpath(out):
                return 100.0
            if p == os.path.normpath(hdr):
                return 200.0
            return 50.0 if os.path.exists(p) else real(p)
        monkeypatch.setattr(os.path, "getmtime", fake)
        assert _build.needs_build(out), hdr
    monkeypatch.setattr(os.path, "getmtime", lambda p: 100.0 if os.path.normpath(p) == os.path.normpath(out) else 50.0)
    assert not _build.needs_build(out)
