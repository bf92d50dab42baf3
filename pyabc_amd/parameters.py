"""Parameter containers (API of pyabc/parameters.py:1-85)."""


class ParameterStructure(dict):
    """dict of parameters; nested dicts are flattened to "a.b" keys."""

    @staticmethod
    def flatten_dict(dict_: dict):
        out = {}
        for key, value in dict_.items():
            if isinstance(value, dict):
                for k2, v2 in ParameterStructure.flatten_dict(value).items():
                    out[f"{key}.{k2}"] = v2
            else:
                out[key] = value
        return out

    def __init__(self, *args, **kwargs):
        if args and kwargs:
            raise Exception("Only keyword or dictionary allowed")
        src = args[0] if args else kwargs
        super().__init__(ParameterStructure.flatten_dict(src) if src else {})


class Parameter(ParameterStructure):
    """A single model parameter; supports key-wise + and - and dot access."""

    def __add__(self, other):
        return Parameter(**{k: self[k] + other[k] for k in self})

    def __sub__(self, other):
        return Parameter(**{k: self[k] - other[k] for k in self})

    def __getattr__(self, item):
        try:
            return self[item]
        except KeyError:
            raise AttributeError(item)

    def __getstate__(self):
        return dict(self)

    def __setstate__(self, state):
        self.update(state)

    def copy(self):
        return Parameter(**self)
