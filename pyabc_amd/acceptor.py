"""Acceptors (API of pyabc/acceptor/acceptor.py:1-306).  The batch sampler
applies the uniform acceptance d <= eps(t) inside the distance kernel."""


class AcceptorResult(dict):
    def __init__(self, distance, accept, weight=1.0):
        super().__init__(distance=distance, accept=accept, weight=weight)

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError:
            raise AttributeError(key)

    __setattr__ = dict.__setitem__


class Acceptor:
    def __init__(self):
        pass

    def initialize(self, t, get_weighted_distances, distance_function, x_0):
        pass

    def update(self, t, get_weighted_distances, prev_temp, acceptance_rate):
        pass

    def __call__(self, distance_function, eps, x, x_0, t, par):
        raise NotImplementedError()

    def get_epsilon_config(self, t):
        return None

    @staticmethod
    def assert_acceptor(maybe_acceptor):
        return SimpleFunctionAcceptor.assert_acceptor(maybe_acceptor)


class SimpleFunctionAcceptor(Acceptor):
    def __init__(self, fun):
        super().__init__()
        self.fun = fun

    def __call__(self, distance_function, eps, x, x_0, t, par):
        return self.fun(distance_function, eps, x, x_0, t, par)

    @staticmethod
    def assert_acceptor(maybe_acceptor):
        if isinstance(maybe_acceptor, Acceptor):
            return maybe_acceptor
        return SimpleFunctionAcceptor(maybe_acceptor)


def accept_use_current_time(distance_function, eps, x, x_0, t, par):
    """d <= eps(t) (acceptor.py:235-244)."""
    d = distance_function(x, x_0, t, par)
    return AcceptorResult(distance=d, accept=d <= eps(t))


def accept_use_complete_history(distance_function, eps, x, x_0, t, par):
    d = distance_function(x, x_0, t, par)
    accept = d <= eps(t)
    if accept:
        for t_prev in range(0, t):
            try:
                accept = distance_function(x, x_0, t_prev, par) <= eps(t_prev)
                if not accept:
                    break
            except Exception:
                accept = True
    return AcceptorResult(distance=d, accept=accept)


class UniformAcceptor(Acceptor):
    def __init__(self, use_complete_history=False):
        super().__init__()
        self.use_complete_history = use_complete_history

    def __call__(self, distance_function, eps, x, x_0, t, par):
        if self.use_complete_history:
            return accept_use_complete_history(distance_function, eps, x,
                                               x_0, t, par)
        return accept_use_current_time(distance_function, eps, x, x_0, t, par)
