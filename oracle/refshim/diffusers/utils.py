import logging as _logging
from collections import OrderedDict


class BaseOutput(OrderedDict):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        for k, v in self.items():
            object.__setattr__(self, k, v)

    def __getitem__(self, k):
        if isinstance(k, int):
            return list(self.values())[k]
        return super().__getitem__(k)


class logging:  # noqa: N801 - mirrors diffusers.utils.logging
    @staticmethod
    def get_logger(name):
        return _logging.getLogger(name)
