"""Every def of the package, the reference-compatible entry points and the bench scripts is
fully annotated -- the ``disallow_untyped_defs`` half of the reference's mypy gate
(reference pyproject.toml [tool.mypy], .github/workflows/lint.yml ``mypy .``), checked with
``ast`` because mypy is not installed in the build image (CI runs mypy itself)."""
import ast
from pathlib import Path
from typing import List

ROOT = Path(__file__).resolve().parent.parent
TARGETS = ["distributed_training_amd", "src", "bench.py", "bench_lm.py", "__graft_entry__.py"]


def _files() -> List[Path]:
    out: List[Path] = []
    for t in TARGETS:
        p = ROOT / t
        out.extend(sorted(p.rglob("*.py")) if p.is_dir() else [p])
    return out


def _untyped(path: Path) -> List[str]:
    bad = []
    for fn in ast.walk(ast.parse(path.read_text())):
        if not isinstance(fn, (ast.FunctionDef, ast.AsyncFunctionDef)):
            continue
        a = fn.args
        pos = a.posonlyargs + a.args
        missing = [x.arg for i, x in enumerate(pos + a.kwonlyargs)
                   if x.annotation is None and not (i == 0 and x.arg in ("self", "cls"))]
        missing += ["*" + x.arg for x in (a.vararg, a.kwarg) if x is not None and x.annotation is None]
        # mypy accepts an __init__ without '-> None' when some argument is annotated
        if fn.returns is None and not (fn.name == "__init__" and len(pos + a.kwonlyargs) > 1):
            missing.append("return")
        if missing:
            bad.append(f"{path.relative_to(ROOT)}:{fn.lineno} {fn.name}: {', '.join(missing)}")
    return bad


def test_every_def_is_annotated() -> None:
    bad = [b for f in _files() for b in _untyped(f)]
    assert not bad, "unannotated definitions:\n" + "\n".join(bad)
