"""Hydra-compatible configuration system (no hydra / omegaconf dependency).

Reproduces what the reference uses from Hydra 1.3
(``@hydra.main(version_base=None, config_path="../conf", config_name="config")``,
reference src/distributed_trainer.py:243, conf/config.yaml:1-14):

* a primary YAML with a ``defaults`` list of config groups (``model: default``,
  ``train: default``) and ``_self_`` ordering;
* command-line overrides: ``train.batch_size=64`` (set), ``+new.key=1`` (add),
  ``++key=1`` (force add/set), ``~key`` (delete), ``model=mlp2`` (group choice);
* interpolations ``${a.b}``, ``${now:%Y-%m-%d}``, ``${hydra:runtime.output_dir}``,
  ``${hydra:job.name}``, ``${oc.env:VAR,default}``;
* ``hydra.run.dir`` creation and ``hydra.job.chdir`` behaviour;
* attribute access and ``.get(key, default)`` on nodes (reference :256-257).

Values are parsed with ``yaml.safe_load`` (never an unsafe loader).
"""
from __future__ import annotations

import copy
import datetime as _dt
import functools
import os
import re
import sys
from pathlib import Path
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import yaml


class ConfigError(ValueError):
    pass


class ConfigNode(dict):
    """dict with attribute access; nested dicts are ConfigNodes."""

    def __init__(self, *args: Any, **kwargs: Any) -> None:
        super().__init__()
        for k, v in dict(*args, **kwargs).items():
            self[k] = v

    def __setitem__(self, key: Any, value: Any) -> None:
        super().__setitem__(key, _wrap(value))

    def __getattr__(self, item: str) -> Any:
        try:
            return self[item]
        except KeyError as e:
            raise AttributeError(f"config has no key {item!r} (keys: {list(self.keys())})") from e

    def __setattr__(self, key: str, value: Any) -> None:
        self[key] = value

    def __delattr__(self, item: str) -> None:
        del self[item]

    def __deepcopy__(self, memo: Any) -> Any:
        return ConfigNode({k: copy.deepcopy(v, memo) for k, v in self.items()})

    def to_dict(self) -> dict:
        return {k: (v.to_dict() if isinstance(v, ConfigNode) else
                    [x.to_dict() if isinstance(x, ConfigNode) else x for x in v] if isinstance(v, list) else v)
                for k, v in self.items()}

    def select(self, dotted: str, default: Any = None) -> Any:
        node: Any = self
        for part in dotted.split("."):
            if isinstance(node, dict) and part in node:
                node = node[part]
            else:
                return default
        return node

    def to_yaml(self) -> str:
        return yaml.safe_dump(self.to_dict(), sort_keys=False)


def _wrap(v: Any) -> Any:
    if isinstance(v, ConfigNode):
        return v
    if isinstance(v, dict):
        return ConfigNode(v)
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


def merge(base: dict, other: dict) -> ConfigNode:
    """Recursive merge; ``other`` wins."""
    out = ConfigNode(copy.deepcopy(dict(base)))
    for k, v in other.items():
        if k in out and isinstance(out[k], dict) and isinstance(v, dict):
            out[k] = merge(out[k], v)
        else:
            out[k] = copy.deepcopy(v)
    return out


def _load_yaml(path: Path) -> dict:
    with open(path, "r", encoding="utf-8") as f:
        data = yaml.safe_load(f)
    if data is None:
        return {}
    if not isinstance(data, dict):
        raise ConfigError(f"{path}: top level must be a mapping")
    return data


def parse_value(text: str) -> Any:
    """Parse an override value the way Hydra's grammar does for the common cases."""
    if text == "":
        return ""
    try:
        return yaml.safe_load(text)
    except yaml.YAMLError:
        return text


class Override:
    __slots__ = ("key", "value", "op")

    def __init__(self, key: str, value: Any, op: str) -> None:
        self.key, self.value, self.op = key, value, op

    def __repr__(self) -> str:
        return f"Override({self.op}{self.key}={self.value!r})"


_OVR = re.compile(r"^(?P<prefix>\+\+|\+|~)?(?P<key>[A-Za-z_@][\w.\-/@]*)(?:=(?P<val>.*))?$", re.S)


def parse_override(text: str) -> Override:
    m = _OVR.match(text)
    if not m:
        raise ConfigError(f"cannot parse override {text!r}")
    prefix = m.group("prefix") or ""
    key = m.group("key")
    val = m.group("val")
    if prefix == "~":
        return Override(key, None if val is None else parse_value(val), "~")
    if val is None:
        raise ConfigError(f"override {text!r} needs a value (key=value)")
    return Override(key, parse_value(val), prefix or "=")


def _set_dotted(cfg: dict, key: str, value: Any, op: str) -> None:
    parts = key.split(".")
    node = cfg
    for p in parts[:-1]:
        if p not in node or not isinstance(node[p], dict):
            if op == "=" and p not in node:
                raise ConfigError(f"key {key!r} not in config (use +{key}=... to add)")
            node[p] = ConfigNode()
        node = node[p]
    leaf = parts[-1]
    if op == "=" and leaf not in node:
        raise ConfigError(f"key {key!r} not in config (use +{key}=... to add)")
    if op == "+" and leaf in node:
        raise ConfigError(f"key {key!r} already in config (use ++{key}=... to force)")
    node[leaf] = value


def _del_dotted(cfg: dict, key: str) -> None:
    parts = key.split(".")
    node = cfg
    for p in parts[:-1]:
        node = node.get(p)
        if not isinstance(node, dict):
            raise ConfigError(f"cannot delete missing key {key!r}")
    if parts[-1] not in node:
        raise ConfigError(f"cannot delete missing key {key!r}")
    del node[parts[-1]]


def _parse_defaults(defaults: Sequence[Any]) -> List[Tuple[str, Optional[str]]]:
    out: List[Tuple[str, Optional[str]]] = []
    for d in defaults:
        if d == "_self_":
            out.append(("_self_", None))
        elif isinstance(d, str):
            out.append((d, None))  # a plain config file in the same dir
        elif isinstance(d, dict) and len(d) == 1:
            (g, opt), = d.items()
            g = str(g).lstrip("/")
            if g.startswith("override "):
                g = g[len("override "):]
            out.append((g, None if opt is None else str(opt)))
        else:
            raise ConfigError(f"bad defaults entry {d!r}")
    return out


def compose(config_dir: os.PathLike, config_name: str = "config", overrides: Iterable[str] = (),
            runtime: Optional[Dict[str, Any]] = None, resolve: bool = True) -> ConfigNode:
    """Compose ``config_dir/config_name.yaml`` with its defaults list and overrides."""
    config_dir = Path(config_dir)
    primary_path = config_dir / f"{config_name}.yaml"
    if not primary_path.exists():
        raise ConfigError(f"primary config {primary_path} not found")
    primary = _load_yaml(primary_path)
    defaults = _parse_defaults(primary.pop("defaults", []) or [])
    ovrs = [parse_override(o) for o in overrides]
    group_names = {g for g, opt in defaults if g != "_self_" and opt is not None}
    choices = {g: opt for g, opt in defaults if g != "_self_"}
    rest: List[Override] = []
    for o in ovrs:
        if o.op in ("=", "+", "++") and (o.key in group_names or (o.op == "+" and (config_dir / o.key).is_dir())):
            if o.key not in choices:
                defaults.append((o.key, str(o.value)))
            choices[o.key] = str(o.value)
        else:
            rest.append(o)
    if not any(g == "_self_" for g, _ in defaults):
        defaults.append(("_self_", None))  # Hydra 1.1+ default: primary last
    cfg = ConfigNode()
    for g, _ in defaults:
        if g == "_self_":
            cfg = merge(cfg, primary)
            continue
        opt = choices.get(g)
        if opt is None:
            path = config_dir / f"{g}.yaml"
            if path.exists():
                cfg = merge(cfg, _load_yaml(path))
            continue
        path = config_dir / g / f"{opt}.yaml"
        if not path.exists():
            avail = sorted(p.stem for p in (config_dir / g).glob("*.yaml")) if (config_dir / g).is_dir() else []
            raise ConfigError(f"could not find {g}/{opt}.yaml (available: {avail})")
        node = _load_yaml(path)
        pkg = node.pop("# @package", None)  # noqa: F841 - header comments are ignored by yaml anyway
        sub = ConfigNode()
        cur = sub
        parts = g.split("/")
        for p in parts[:-1]:
            cur[p] = ConfigNode()
            cur = cur[p]
        cur[parts[-1]] = node
        cfg = merge(cfg, sub)
    for o in rest:
        if o.op == "~":
            _del_dotted(cfg, o.key)
        else:
            _set_dotted(cfg, o.key, o.value, o.op)
    hydra_node = cfg.get("hydra", ConfigNode())
    hydra_node.setdefault("runtime", ConfigNode())
    hydra_node.setdefault("job", ConfigNode())
    hydra_node["runtime"].update(runtime or {})
    hydra_node["runtime"].setdefault("choices", ConfigNode(choices))
    hydra_node["job"].setdefault("name", Path(sys.argv[0]).stem if sys.argv and sys.argv[0] else "app")
    hydra_node["overrides"] = ConfigNode({"task": list(overrides)})
    cfg["hydra"] = hydra_node
    if resolve:
        cfg = resolve_interpolations(cfg)
    return cfg


_INTERP = re.compile(r"\$\{([^${}]+)\}")


def _now_str(fmt: str) -> str:
    stamp = os.environ.get("DTA_RUN_TIMESTAMP")  # shared across ranks when set by the launcher
    t = _dt.datetime.fromtimestamp(float(stamp)) if stamp else _NOW
    return t.strftime(fmt)


_NOW = _dt.datetime.now()


def _resolve_expr(expr: str, root: ConfigNode, stack: Tuple[str, ...]) -> Any:
    expr = expr.strip()
    if expr.startswith("now:"):
        return _now_str(expr[4:])
    if expr.startswith("oc.env:"):
        body = expr[len("oc.env:"):]
        name, _, default = body.partition(",")
        val = os.environ.get(name.strip())
        if val is None:
            if not _:
                raise ConfigError(f"environment variable {name!r} not set")
            return parse_value(default.strip())
        return val
    if expr.startswith("hydra:"):
        key = "hydra." + expr[len("hydra:"):]
    else:
        key = expr
    if key in stack:
        raise ConfigError(f"interpolation cycle at ${{{expr}}}")
    val = root.select(key, _MISSING)
    if val is _MISSING:
        raise ConfigError(f"interpolation ${{{expr}}} refers to a missing key")
    return _resolve_value(val, root, stack + (key,))


_MISSING = object()


def _resolve_value(v: Any, root: ConfigNode, stack: Tuple[str, ...]) -> Any:
    if isinstance(v, str):
        m = _INTERP.fullmatch(v)
        if m:
            return _resolve_expr(m.group(1), root, stack)
        if "${" in v:
            return _INTERP.sub(lambda mm: str(_resolve_expr(mm.group(1), root, stack)), v)
        return v
    if isinstance(v, dict):
        return ConfigNode({k: _resolve_value(x, root, stack) for k, x in v.items()})
    if isinstance(v, list):
        return [_resolve_value(x, root, stack) for x in v]
    return v


def resolve_interpolations(cfg: ConfigNode) -> ConfigNode:
    # resolve hydra.run.dir first so ${hydra:runtime.output_dir} can default to it
    hyd = cfg.get("hydra", ConfigNode())
    run_dir = hyd.select("run.dir")
    if run_dir is not None and "output_dir" not in hyd["runtime"]:
        hyd["runtime"]["output_dir"] = str(Path(_resolve_value(run_dir, cfg, ())).absolute())
    elif "output_dir" not in hyd["runtime"]:
        hyd["runtime"]["output_dir"] = os.getcwd()
    return _resolve_value(cfg, cfg, ())


def split_argv(argv: Sequence[str]) -> Tuple[List[str], List[str]]:
    """Split ``argv`` into (hydra-style overrides, other args)."""
    ovr, other = [], []
    for a in argv:
        if not a.startswith("-") and ("=" in a or a.startswith("~")):
            ovr.append(a)
        elif a.startswith("+") and "=" in a:
            ovr.append(a)
        else:
            other.append(a)
    return ovr, other


def prepare_run_dir(cfg: ConfigNode) -> Path:
    """Create hydra.runtime.output_dir, write .hydra/config.yaml, chdir if
    hydra.job.chdir (reference conf/config.yaml:10-14)."""
    out = Path(cfg.hydra.runtime.output_dir)
    out.mkdir(parents=True, exist_ok=True)
    meta = out / ".hydra"
    meta.mkdir(exist_ok=True)
    try:
        body = {k: v for k, v in cfg.to_dict().items() if k != "hydra"}
        (meta / "config.yaml").write_text(yaml.safe_dump(body, sort_keys=False))
        (meta / "overrides.yaml").write_text(yaml.safe_dump(list(cfg.hydra.overrides.task)))
    except OSError:
        pass
    if cfg.select("hydra.job.chdir", False):
        os.chdir(out)
    return out


def main_decorator(config_path: str, config_name: str, version_base: Optional[str] = None) -> Callable:
    """Drop-in for ``@hydra.main``: composes the config from ``sys.argv`` and
    calls the task function with it."""

    def deco(fn: Callable[[ConfigNode], Any]) -> Any:
        @functools.wraps(fn)
        def wrapper(cfg_passthrough: Optional[ConfigNode] = None, argv: Optional[Sequence[str]] = None) -> Any:
            if cfg_passthrough is not None:
                return fn(cfg_passthrough)
            src = Path(sys.modules[fn.__module__].__file__).resolve().parent
            cdir = (src / config_path).resolve() if not os.path.isabs(config_path) else Path(config_path)
            args = list(sys.argv[1:] if argv is None else argv)
            ovr, other = split_argv(args)
            if other:
                raise SystemExit(f"unrecognised arguments: {other}")
            cfg = compose(cdir, config_name, ovr, runtime={"cwd": os.getcwd(), "config_dir": str(cdir)})
            prepare_run_dir(cfg)
            return fn(cfg)

        return wrapper

    return deco
