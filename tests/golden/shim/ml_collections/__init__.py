"""Minimal ConfigDict (attribute access over nested dicts; test shim)."""


class ConfigDict(dict):
    def __init__(self, d=None, **kw):
        super().__init__()
        for k, v in dict(d or {}, **kw).items():
            self[k] = ConfigDict(v) if isinstance(v, dict) and not isinstance(v, ConfigDict) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v
