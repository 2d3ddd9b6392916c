import functools
import inspect


class _AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


class FrozenDict(_AttrDict):
    pass


class ConfigMixin:
    @classmethod
    def from_config(cls, config):
        return cls(**dict(config))


def register_to_config(init):
    sig = inspect.signature(init)

    @functools.wraps(init)
    def wrapper(self, *args, **kwargs):
        bound = sig.bind(self, *args, **kwargs)
        bound.apply_defaults()
        cfg = dict(bound.arguments)
        cfg.pop("self")
        init(self, *args, **kwargs)
        self._internal_dict = FrozenDict(cfg)

    return wrapper
