"""Typed, JSON-serialisable stage parameters (Flink-ML ``ParamInfo`` / ``Params`` /
``WithParams``) and the reference's parameter mixins.

Same parameter NAMES, descriptions, required/optional flags and defaults as
``param/*.java`` (e.g. ``HasClusterConfig.java:14-53``: ``zookeeper_connect_str`` default
``127.0.0.1:2181``, ``worker_num`` 1, ``ps_num`` 0).  Every mixin contributes fluent
``set_x(v) -> self`` / ``get_x()`` accessors plus the Java-style ``setX``/``getX`` aliases,
so code written against the reference's API reads the same.

``Params.to_json`` follows Flink-ML's layout: a JSON object mapping each parameter name
to the JSON encoding of its value; ``load_json`` overlays onto existing values
(``App.java:125-127``).
"""
from __future__ import annotations

import enum
import json
from typing import Any, Dict, Iterable, Optional

_MISSING = object()


class ParamInfo:
    def __init__(self, name: str, value_class: type, description: str = "", required: bool = False,
                 default: Any = _MISSING, alias: Iterable[str] = ()):
        self.name = name
        self.value_class = value_class
        self.description = description
        self.is_optional = not required
        self.has_default_value = default is not _MISSING
        self.default_value = None if default is _MISSING else default
        self.alias = tuple(alias)

    def __repr__(self):
        return f"ParamInfo({self.name!r}, {self.value_class.__name__})"


def _to_jsonable(v):
    if isinstance(v, enum.Enum):
        return v.name
    if isinstance(v, (list, tuple)):
        return [_to_jsonable(x) for x in v]
    return v


class Params:
    def __init__(self):
        self._m: Dict[str, str] = {}  # name -> JSON-encoded value (Flink-ML layout)

    # ------------------------------------------------------------------ access
    def get(self, info: ParamInfo):
        for name in (info.name, *info.alias):
            if name in self._m:
                return _decode(info, json.loads(self._m[name]))
        if info.has_default_value:
            return info.default_value
        if not info.is_optional:
            raise ValueError(f"Missing non-optional parameter {info.name}")
        return None

    def set(self, info: ParamInfo, value) -> "Params":
        self._m[info.name] = json.dumps(_to_jsonable(value))
        return self

    def remove(self, info: ParamInfo) -> None:
        self._m.pop(info.name, None)

    def contains(self, info: ParamInfo) -> bool:
        return info.name in self._m or any(a in self._m for a in info.alias)

    def size(self) -> int:
        return len(self._m)

    def is_empty(self) -> bool:
        return not self._m

    def clear(self) -> None:
        self._m.clear()

    def clone(self) -> "Params":
        p = Params()
        p._m = dict(self._m)
        return p

    def merge(self, other: "Params") -> "Params":
        self._m.update(other._m)
        return self

    # ------------------------------------------------------------------ JSON
    def to_json(self) -> str:
        return json.dumps(self._m, sort_keys=True)

    def load_json(self, s: str) -> "Params":
        m = json.loads(s)
        if not isinstance(m, dict):
            raise ValueError("Params JSON must be an object")
        for k, v in m.items():
            self._m[k] = v if isinstance(v, str) else json.dumps(v)
        return self

    @classmethod
    def from_json(cls, s: str) -> "Params":
        return cls().load_json(s)

    toJson, loadJson, fromJson = to_json, load_json, from_json

    def __eq__(self, o):
        return isinstance(o, Params) and self._m == o._m

    def __repr__(self):
        return f"Params({self._m})"


def _decode(info: ParamInfo, v):
    vc = info.value_class
    if v is None:
        return None
    if isinstance(vc, type) and issubclass(vc, enum.Enum):
        return vc[v]
    if vc is list and info.name.endswith("Types"):
        from .types import DataTypes
        return [DataTypes[x] for x in v]
    if vc is list:
        return list(v)
    return vc(v)


class WithParams:
    """Fluent parameter access (Flink-ML ``WithParams``)."""

    def get_params(self) -> Params:
        if not hasattr(self, "_params"):
            self._params = Params()
        return self._params

    getParams = get_params

    def set(self, info: ParamInfo, value):
        self.get_params().set(info, value)
        return self

    def get(self, info: ParamInfo):
        return self.get_params().get(info)


def _camel(s: str) -> str:
    parts = s.split("_")
    return parts[0][:1].upper() + parts[0][1:] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def _accessors(cls, info: ParamInfo, short: str, camel: Optional[str] = None):
    """Attach set_<short>/get_<short> (+ setX/getX Java-style aliases) to a mixin."""
    def setter(self, v, _i=info):
        return self.set(_i, v)

    def getter(self, _i=info):
        return self.get(_i)
    setattr(cls, f"set_{short}", setter)
    setattr(cls, f"get_{short}", getter)
    c = camel or _camel(short)
    setattr(cls, f"set{c}", setter)
    setattr(cls, f"get{c}", getter)


# ---------------------------------------------------------------------- mixins
class HasClusterConfig(WithParams):
    """HasClusterConfig.java:14-53.  ZooKeeper is replaced by a torch.distributed TCPStore
    rendezvous: ``WorkerJob`` (api/worker.py) starts every worker on this host with
    MASTER_ADDR=127.0.0.1 and a free port.  The connect string is kept for API and JSON parity
    only; it is not used to locate the rendezvous."""
    ZOOKEEPER_CONNECT_STR = ParamInfo("zookeeper_connect_str", str, "zookeeper address to connect", True,
                                      "127.0.0.1:2181")
    WORKER_NUM = ParamInfo("worker_num", int, "worker number", True, 1)
    PS_NUM = ParamInfo("ps_num", int, "ps number", True, 0)


_accessors(HasClusterConfig, HasClusterConfig.ZOOKEEPER_CONNECT_STR, "zookeeper_conn_str", "ZookeeperConnStr")
_accessors(HasClusterConfig, HasClusterConfig.WORKER_NUM, "worker_num")
_accessors(HasClusterConfig, HasClusterConfig.PS_NUM, "ps_num")


def _python_config(prefix: str, what: str):
    class _M(WithParams):
        pass
    scripts = ParamInfo(f"{prefix}_scripts", list,
                        f"python scripts path, the first file entry, for {what} processing", True)
    func = ParamInfo(f"{prefix}_map_func", str, f"the entry function in entry file to be called, for {what} processing",
                     True)
    key = ParamInfo(f"{prefix}_hyper_params_key", str,
                    f"the key name to get hyper params from context inf TensorFlow, for {what} processing", True)
    hp = ParamInfo(f"{prefix}_hyper_params", list,
                   f"hyper params for TensorFlow, each param format is '--param1=value1', for {what} processing",
                   True, [])
    env = ParamInfo(f"{prefix}_env_path", str, f"virtual environment path, for {what} processing", False, None)
    P = prefix.upper()
    for attr, info in ((f"{P}_SCRIPTS", scripts), (f"{P}_MAP_FUNC", func), (f"{P}_HYPER_PARAMS_KEY", key),
                       (f"{P}_HYPER_PARAMS", hp), (f"{P}_ENV_PATH", env)):
        setattr(_M, attr, info)
        _accessors(_M, info, info.name)
    return _M


class HasTrainPythonConfig(_python_config("train", "train")):
    """HasTrainPythonConfig.java:16-79."""


class HasInferencePythonConfig(_python_config("inference", "inference")):
    """HasInferencePythonConfig.java:16-79."""


def _cols(name: str, desc: str, vc=list):
    class _M(WithParams):
        pass
    info = ParamInfo(name, vc, desc, True)
    setattr(_M, "".join("_" + c if c.isupper() else c.upper() for c in name).upper().lstrip("_"), info)
    snake = "".join("_" + c.lower() if c.isupper() else c for c in name)
    _accessors(_M, info, snake, name[:1].upper() + name[1:])
    return _M


class HasTrainSelectedCols(_cols("trainSelectedCols", "Names of the columns used for train processing")):
    """HasTrainSelectedCols.java:11-24."""


class HasTrainOutputCols(_cols("trainOutputCols", "Names of the output columns for train processing")):
    """HasTrainOutputCols.java:11-24."""


class HasTrainOutputTypes(_cols("trainOutputTypes", "TypeInformation of output columns for train processing")):
    """HasTrainOutputTypes.java:12-25 (values are ``DataTypes``)."""


class HasInferenceSelectedCols(_cols("inferenceSelectedCols", "Names of the columns used for inference processing")):
    """HasInferenceSelectedCols.java:11-24."""


class HasInferenceOutputCols(_cols("inferenceOutputCols", "Names of the output columns for inference processing")):
    """HasInferenceOutputCols.java:11-24."""


class HasInferenceOutputTypes(_cols("inferenceOutputTypes",
                                    "TypeInformation of output columns for inference processing")):
    """HasInferenceOutputTypes.java:12-25 (values are ``DataTypes``)."""
