"""Every measurement the documentation cites exists: the profile files named in README.md, CHANGELOG.md,
docs/*.md and profiles/*.md (r<round>_... names, with or without the profiles/ prefix) and the BENCH
records it quotes are in the tree, so each number traces to a file."""
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
NAME = re.compile(r"(?<![\w{,/.-])(?:profiles/)?(r\d+_[A-Za-z0-9_.\-]+?\.(?:txt|json|csv|md))(?![\w{}])")


def _docs():
    yield ROOT / "README.md"
    yield ROOT / "CHANGELOG.md"
    yield from sorted((ROOT / "docs").glob("*.md"))
    yield from sorted((ROOT / "profiles").glob("*.md"))


def test_cited_profiles_exist():
    missing = []
    for doc in _docs():
        for m in NAME.finditer(doc.read_text()):
            name = m.group(1)
            if not (ROOT / "profiles" / name).exists() and not (ROOT / name).exists():
                missing.append(f"{doc.relative_to(ROOT)}: {name}")
    assert not missing, "cited but absent: " + ", ".join(sorted(set(missing)))


def test_readme_stays_short():
    assert len((ROOT / "README.md").read_text().splitlines()) <= 200
