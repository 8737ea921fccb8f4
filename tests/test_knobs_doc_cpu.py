"""docs/KNOBS.md stays honest in both directions: every ``LUMEN_*`` variable it documents is read
somewhere in the package, the tools or bench.py (a renamed or removed knob fails here), and every
variable the package reads is documented (an undocumented A/B switch fails here)."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
_SUFFIXES = {".py", ".hip", ".cpp", ".h", ".sh"}


def _sources() -> str:
    out = [(ROOT / "bench.py").read_text()]
    for d in ("lumen_amd", "tools"):
        for p in (ROOT / d).rglob("*"):
            if p.is_file() and p.suffix in _SUFFIXES:
                out.append(p.read_text(errors="ignore"))
    return "\n".join(out)


def test_documented_knobs_exist():
    doc = (ROOT / "docs" / "KNOBS.md").read_text()
    names = set(re.findall(r"`(LUMEN_[A-Z0-9_]+)`", doc))
    assert len(names) > 20
    src = _sources()
    missing = sorted(n for n in names if n not in src)
    assert not missing, f"documented but never read: {missing}"


def test_every_read_knob_is_documented():
    doc = (ROOT / "docs" / "KNOBS.md").read_text()
    names = set(re.findall(r"`(LUMEN_[A-Z0-9_]+)`", doc))
    pat = re.compile(r'(?:environ\.get\(|environ\[|getenv\()\s*"(LUMEN_[A-Z0-9_]+)"')
    undocumented = set()
    for p in (ROOT / "lumen_amd").rglob("*"):
        if p.is_file() and p.suffix in _SUFFIXES:
            undocumented |= {m.group(1) for m in pat.finditer(p.read_text(errors="ignore"))} - names
    assert not undocumented, f"read but not in docs/KNOBS.md: {sorted(undocumented)}"
