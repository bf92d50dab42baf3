"""Sequential sampler (API of pyabc/sampler/singlecore.py:1-38).

Semantics the reference defines there, restated as one evaluation loop:
every call of ``simulate_one`` is one evaluation and is counted; with
``check_max_eval`` no evaluation starts once ``max_eval`` of them have run;
the loop ends at the n-th acceptance; a sample that ends short of n
acceptances is marked ``ok = False``.  (The reference nests a per-particle
loop inside a loop over n; both stop at the same evaluation.)
"""
import numpy as np

from .base import Sampler


class SingleCoreSampler(Sampler):
    def __init__(self, check_max_eval=False):
        super().__init__()
        self.check_max_eval = check_max_eval

    def _may_start(self, done, max_eval):
        return not self.check_max_eval or done < max_eval

    def sample_until_n_accepted(self, n, simulate_one, max_eval=np.inf,
                                all_accepted=False):
        sample = self._create_empty_sample()
        done = accepted = 0
        while accepted < n and self._may_start(done, max_eval):
            particle = simulate_one()
            done += 1
            accepted += bool(particle.accepted)
            sample.append(particle)
        self.nr_evaluations_ = done
        sample.ok = sample.ok and accepted >= n
        return sample
