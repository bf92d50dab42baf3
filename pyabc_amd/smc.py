"""ABCSMC with the reference's API (pyabc/smc.py:24-1061), MI355X back end.

The generation loop, the per-proposal closure and the between-generation
updates follow the reference's control flow (file:line cited per method).
The difference is the batch hook: ``_create_simulate_function`` attaches a
:class:`~pyabc_amd.sampler.gpu.BatchSpec` to the closure, so the default
:class:`GPUBatchSampler` runs the generation as HIP kernels on the device,
and populations stay on the device as columns between generations.
"""
import copy
import datetime
import time
import logging

import numpy as np
import pandas as pd
import torch

from .acceptor import UniformAcceptor, SimpleFunctionAcceptor
from .distance import PNormDistance, to_distance
from .epsilon import MedianEpsilon
from .model import SimpleModel
from .parameters import Parameter
from .population import Particle, ColumnarPopulation, DistanceToGroundTruth
from .populationstrategy import ConstantPopulationSize
from .random_variables import RV, ModelPerturbationKernel
from .sampler import GPUBatchSampler
from .sampler.gpu import BatchSpec
from .storage import History
from .transition import MultivariateNormalTransition
from .temperature import DeviceRecords, TemperatureBase
from .weighted_statistics import effective_sample_size

logger = logging.getLogger("ABC")


def identity(x):
    return x


def fast_random_choice(weights):
    """Index drawn from (unnormalised-safe) weights by one uniform
    (pyabc_rand_choice.py:4-17)."""
    cs = 0
    u = np.random.rand()
    for k, w in enumerate(weights):
        cs += w
        if u <= cs:
            return k
    raise Exception(f"Random choice error {weights}")


class ABCSMC:
    """Approximate Bayesian computation by sequential Monte Carlo."""

    def __init__(self, models, parameter_priors, distance_function=None,
                 population_size=100, summary_statistics=identity,
                 model_prior=None, model_perturbation_kernel=None,
                 transitions=None, eps=None, sampler=None, acceptor=None,
                 stop_if_only_single_model_alive=False,
                 max_nr_recorded_particles=np.inf):
        if not isinstance(models, list):
            models = [models]
        self.models = list(map(SimpleModel.assert_model, models))
        if not isinstance(parameter_priors, list):
            parameter_priors = [parameter_priors]
        self.parameter_priors = parameter_priors
        if len(self.models) != len(self.parameter_priors):
            raise AssertionError(
                "Number models and number parameter priors have to agree.")
        if distance_function is None:
            distance_function = PNormDistance()
        self.distance_function = to_distance(distance_function)
        self.summary_statistics = summary_statistics
        if model_prior is None:
            model_prior = RV("randint", 0, len(self.models))
        self.model_prior = model_prior
        if model_perturbation_kernel is None:
            model_perturbation_kernel = ModelPerturbationKernel(
                len(self.models), probability_to_stay=.7)
        self.model_perturbation_kernel = model_perturbation_kernel
        if transitions is None:
            transitions = [MultivariateNormalTransition()
                           for _ in self.models]
        if not isinstance(transitions, list):
            transitions = [transitions]
        self.transitions = transitions
        if eps is None:
            eps = MedianEpsilon(median_multiplier=1)
        self.eps = eps
        if isinstance(population_size, int):
            population_size = ConstantPopulationSize(population_size)
        self.population_size = population_size
        if sampler is None:
            sampler = GPUBatchSampler()
        self.sampler = sampler
        if acceptor is None:
            acceptor = UniformAcceptor()
        self.acceptor = SimpleFunctionAcceptor.assert_acceptor(acceptor)
        self.stop_if_only_single_model_alive = stop_if_only_single_model_alive
        self.max_nr_recorded_particles = max_nr_recorded_particles
        self.x_0 = None
        self.history = None
        self._initial_population = None
        self.minimum_epsilon = None
        self.max_nr_populations = None
        self.min_acceptance_rate = None
        self.generation_log = []

    def __getstate__(self):
        state = self.__dict__.copy()
        del state["sampler"]
        return state

    # ------------------------------------------------------------------
    def new(self, db, observed_sum_stat=None, *, gt_model=None, gt_par=None,
            meta_info=None):
        """Start a run (smc.py:248-346).  ``db``: ``"sqlite:///file.db"``
        (the reference's SQL schema on disk), ``"sqlite://"`` (the same in
        memory) or any other id (device populations only, no SQL)."""
        self.x_0 = {} if observed_sum_stat is None else observed_sum_stat
        self.history = History(db)
        self.history.store_initial_data(
            gt_model, meta_info, self.x_0, gt_par or {},
            [m.name for m in self.models], self.distance_function.to_json(),
            self.eps.to_json(), self.population_size.to_json())
        return self.history

    def load(self, db, abc_id=1, observed_sum_stat=None):
        """Continue a run (smc.py:348-382): one held in this process, or one
        stored in a ``sqlite:///file.db`` History (this package's or the
        reference's; the next fit then reads the last population from the
        file)."""
        h = History.lookup(db)
        if h is None or h.id != abc_id:
            if not db.startswith("sqlite:///"):
                raise ValueError(f"no in-memory history {db!r} in this "
                                 "process")
            h = History(db, _id=abc_id, create=False)
        self.history = h
        self.history.id = abc_id
        self.x_0 = observed_sum_stat if observed_sum_stat is not None \
            else h.observed_sum_stat()
        return self.history

    # ------------------------------------------------------------------
    def _initialize_dist_eps_acc(self, t):
        """smc.py:384-445."""
        def get_initial_sum_stats():
            return self._get_initial_population(t).get_accepted_sum_stats()

        def _pop_with_distances():
            pop = self._get_initial_population(t)
            self._update_distances(pop, t)
            return pop

        def get_initial_weighted_distances():
            return _pop_with_distances().get_weighted_distances()

        self.distance_function.initialize(t, get_initial_sum_stats, self.x_0)
        self.acceptor.initialize(t, get_initial_weighted_distances,
                                 self.distance_function, self.x_0)

        def get_initial_records():
            pop = _pop_with_distances()
            if isinstance(pop, ColumnarPopulation):
                # dummy densities 1 (only their quotient matters)
                zero = torch.zeros_like(pop.d)
                return DeviceRecords(pop.d, zero, zero, zero + 1.0)
            return [{"distance": d, "transition_pd_prev": 1.0,
                     "transition_pd": 1.0, "accepted": True}
                    for p in pop.get_list() for d in p.accepted_distances]

        self.eps.initialize(t, get_initial_weighted_distances,
                            get_initial_records, self.max_nr_populations,
                            self.acceptor.get_epsilon_config(t))

    def _update_distances(self, population, t):
        # smc.py:978-984; a device population runs the distance's batch
        # kernel when it has one
        population.update_distances(
            DistanceToGroundTruth(self.distance_function, self.x_0, t))

    def _get_initial_population(self, t):
        """smc.py:447-470 (cached)."""
        if self._initial_population is None:
            if self.history.n_populations > 0:
                self._initial_population = self.history.get_population()
            else:
                self._initial_population = self._sample_from_prior(t)
                self.history.update_nr_samples(
                    History.PRE_TIME, self.sampler.nr_evaluations_)
        return self._initial_population

    def _spec(self, t, kind):
        mp = None
        if t > 0:
            mp = self.history.model_probabilities_dict(t - 1)
        return BatchSpec(t, kind, self.models, self.parameter_priors,
                         self.transitions, self.distance_function, self.eps,
                         self.acceptor, self.x_0,
                         self.population_size.nr_samples_per_parameter,
                         self.summary_statistics, mp)

    def _create_simulate_from_prior_function(self, t):
        """smc.py:472-514."""
        model_prior = self.model_prior
        priors = self.parameter_priors
        models = self.models
        summary_statistics = self.summary_statistics

        def simulate_one():
            m = int(model_prior.rvs())
            theta = priors[m].rvs()
            res = models[m].summary_statistics(t, theta, summary_statistics)
            return Particle(m=m, parameter=theta, weight=1.0,
                            accepted_sum_stats=[res.sum_stats],
                            accepted_distances=[np.inf],
                            rejected_sum_stats=[], rejected_distances=[],
                            accepted=True)

        simulate_one.batch_spec = self._spec(t, "calibration")
        return simulate_one

    def _sample_from_prior(self, t):
        """smc.py:516-534."""
        simulate_one = self._create_simulate_from_prior_function(t)
        logger.info(f"Calibration sample before t={t}.")
        sample = self.sampler.sample_until_n_accepted(
            self.population_size(-1), simulate_one, max_eval=np.inf,
            all_accepted=True)
        return sample.get_accepted_population()

    def _create_simulate_function(self, t):
        """Per-proposal closure (smc.py:536-600) with the batch spec."""
        mp = self.history.model_probabilities_dict(t - 1)
        m = np.array(list(mp.keys()))
        p = np.array(list(mp.values()), dtype=np.float64)
        model_prior = self.model_prior
        priors = self.parameter_priors
        mpk = self.model_perturbation_kernel
        transitions = self.transitions
        nrs = self.population_size.nr_samples_per_parameter
        models = self.models
        summary_statistics = self.summary_statistics
        distance_function = self.distance_function
        eps = self.eps
        acceptor = self.acceptor
        x_0 = self.x_0
        weight_function = self._create_weight_function(t)

        def simulate_one():
            par = ABCSMC._generate_valid_proposal(t, m, p, model_prior,
                                                  priors, mpk, transitions)
            return ABCSMC._evaluate_proposal(*par, t, nrs, models,
                                             summary_statistics,
                                             distance_function, eps, acceptor,
                                             x_0, weight_function)

        simulate_one.batch_spec = self._spec(t, "smc")
        return simulate_one

    @staticmethod
    def _generate_valid_proposal(t, m, p, model_prior, parameter_priors,
                                 model_perturbation_kernel, transitions):
        """smc.py:602-645: resample/perturb until prior-supported."""
        if t == 0:
            m_ss = int(model_prior.rvs())
            return m_ss, parameter_priors[m_ss].rvs()
        while True:
            if len(m) > 1:
                m_s = m[fast_random_choice(p)]
                m_ss = model_perturbation_kernel.rvs(m_s)
                if m_ss not in m:
                    continue
            else:
                m_ss = m[0]
            theta_ss = transitions[m_ss].rvs()
            if model_prior.pmf(m_ss) * parameter_priors[m_ss].pdf(theta_ss) > 0:
                return m_ss, theta_ss

    @staticmethod
    def _evaluate_proposal(m_ss, theta_ss, t, nr_samples_per_parameter,
                           models, summary_statistics, distance_function, eps,
                           acceptor, x_0, weight_function):
        """smc.py:647-707."""
        acc_ss, acc_d, rej_ss, rej_d, acc_w = [], [], [], [], []
        for _ in range(nr_samples_per_parameter):
            r = models[m_ss].accept(t, theta_ss, summary_statistics,
                                    distance_function, eps, acceptor, x_0)
            if r.accepted:
                acc_ss.append(r.sum_stats)
                acc_d.append(r.distance)
                acc_w.append(r.weight)
            else:
                rej_ss.append(r.sum_stats)
                rej_d.append(r.distance)
        accepted = len(acc_ss) > 0
        weight = weight_function(acc_d, m_ss, theta_ss, acc_w) \
            if accepted else 0
        return Particle(m=m_ss, parameter=theta_ss, weight=weight,
                        accepted_sum_stats=acc_ss, accepted_distances=acc_d,
                        rejected_sum_stats=rej_ss, rejected_distances=rej_d,
                        accepted=accepted)

    def _create_transition_pdf(self, t, transitions=None):
        """smc.py:709-733 (density through the device KDE)."""
        if t == 0:
            return self._create_prior_pdf()
        mp = self.history.get_model_probabilities(t - 1)
        mpk = self.model_perturbation_kernel
        transitions = transitions if transitions is not None \
            else self.transitions

        def transition_pdf(m_ss, theta_ss):
            model_factor = sum(row.p * mpk.pmf(m_ss, m)
                               for m, row in mp.iterrows())
            particle_factor = transitions[m_ss].pdf(pd.Series(dict(theta_ss)))
            tpd = model_factor * particle_factor
            if tpd == 0:
                logger.debug("Transition density is zero!")
            return tpd
        return transition_pdf

    def _create_prior_pdf(self):
        model_prior = self.model_prior
        priors = self.parameter_priors

        def prior_pdf(m_ss, theta_ss):
            return model_prior.pmf(m_ss) * priors[m_ss].pdf(theta_ss)
        return prior_pdf

    def _create_weight_function(self, t):
        """smc.py:735-794."""
        nrs = self.population_size.nr_samples_per_parameter
        if t == 0:
            def prior_weight_function(distance_list, m_ss, theta_ss,
                                      acceptance_weights):
                return len(distance_list) / nrs * np.prod(acceptance_weights)
            return prior_weight_function
        transition_pdf = self._create_transition_pdf(t)
        prior_pdf = self._create_prior_pdf()

        def weight_function(distance_list, m_ss, theta_ss, acceptance_weights):
            return (prior_pdf(m_ss, theta_ss) * np.prod(acceptance_weights)
                    * (len(distance_list) / nrs)
                    / transition_pdf(m_ss, theta_ss))
        return weight_function

    # ------------------------------------------------------------------
    def run(self, minimum_epsilon=None, max_nr_populations=np.inf,
            min_acceptance_rate=0.):
        """Generation loop (smc.py:796-940)."""
        if minimum_epsilon is None:
            # a temperature schedule stops at T = 1 (smc.py:843-847)
            minimum_epsilon = 1.0 if isinstance(self.eps, TemperatureBase) \
                else 0.0
        self.minimum_epsilon = minimum_epsilon
        self.max_nr_populations = max_nr_populations
        self.min_acceptance_rate = min_acceptance_rate
        t0 = self.history.max_t + 1
        self.history.start_time = datetime.datetime.now()
        self._fit_transitions(t0)
        self._adapt_population_size(t0)
        self._initialize_dist_eps_acc(t0)
        self.distance_function.configure_sampler(self.sampler)
        self.eps.configure_sampler(self.sampler)
        t_max = t0 + max_nr_populations - 1
        t = t0
        while t <= t_max:
            current_eps = self.eps(t)
            logger.info(f"t: {t}, eps: {current_eps}.")
            simulate_one = self._create_simulate_function(t)
            pop_size = self.population_size(t)
            max_eval = np.inf if min_acceptance_rate == 0. \
                else pop_size / min_acceptance_rate
            t_start = datetime.datetime.now()
            started = time.perf_counter()
            sample = self.sampler.sample_until_n_accepted(
                pop_size, simulate_one, max_eval)
            sample_s = (datetime.datetime.now() - t_start).total_seconds()
            if not sample.ok:
                logger.info("Stopping: sample not ok.")
                break
            population = sample.get_accepted_population()
            n_sim = self.sampler.nr_evaluations_
            self.history.append_population(
                t, current_eps, population, n_sim,
                [m.name for m in self.models])
            pop_size = len(population)
            acceptance_rate = pop_size / n_sim
            wd = population.get_weighted_distances()
            ess = effective_sample_size(
                wd.w_tensor if hasattr(wd, "w_tensor") else wd["w"])
            logger.info(f"Acceptance rate: {pop_size} / {n_sim} = "
                        f"{acceptance_rate:.4e}, ESS={ess:.4e}.")
            self.generation_log.append(dict(
                t=t, eps=current_eps, n_sim=n_sim, ess=ess,
                sample_seconds=sample_s, started=started,
                batch=getattr(self.sampler, "fallback_reason", "") is None))
            self._prepare_next_iteration(t + 1, sample, population,
                                         acceptance_rate)
            if current_eps <= self.minimum_epsilon:
                logger.info("Stopping: minimum epsilon.")
                break
            elif self.stop_if_only_single_model_alive and \
                    self.history.nr_of_models_alive() <= 1:
                logger.info("Stopping: single model alive.")
                break
            elif acceptance_rate < min_acceptance_rate:
                logger.info("Stopping: minimum acceptance rate.")
                break
            t += 1
        self.history.done()
        return self.history

    def _prepare_next_iteration(self, t, sample, population, acceptance_rate):
        """smc.py:942-1022."""
        prev_transitions = [copy.copy(tr) for tr in self.transitions]
        self._fit_transitions(t)
        self._adapt_population_size(t)

        def get_recorded_sum_stats():
            return sample.first_m_sum_stats(self.max_nr_recorded_particles)

        df_updated = self.distance_function.update(t, get_recorded_sum_stats)

        def get_weighted_distances():
            if df_updated:
                self._update_distances(population, t)
            return population.get_weighted_distances()

        self.acceptor.update(t, get_weighted_distances, self.eps(t - 1),
                             acceptance_rate)

        def get_all_records():
            if getattr(sample, "rec_particles", None) is not None:
                return self._device_records(t, sample, prev_transitions)
            recorded = sample.first_m_particles(self.max_nr_recorded_particles)
            tp_prev = self._create_transition_pdf(t - 1, prev_transitions)
            tp = self._create_transition_pdf(t)
            records = []
            for particle in recorded:
                a = tp_prev(particle.m, particle.parameter)
                b = tp(particle.m, particle.parameter)
                for d in (particle.accepted_distances
                          + particle.rejected_distances):
                    records.append({"distance": d, "transition_pd_prev": a,
                                    "transition_pd": b,
                                    "accepted": particle.accepted})
            return records

        self.eps.update(t, get_weighted_distances, get_all_records,
                        acceptance_rate, self.acceptor.get_epsilon_config(t))

    def _device_records(self, t, sample, prev_transitions):
        """get_all_records of a device generation (smc.py:990-1017): the
        previous and current transition log-densities of every recorded
        evaluation by the device KDE pass (or the prior's, at t - 1 = 0)."""
        theta, d, acc = sample.rec_particles[:3]
        parent = sample.rec_particles[3] if len(sample.rec_particles) > 3 \
            else None
        m = int(self.max_nr_recorded_particles) if np.isfinite(
            self.max_nr_recorded_particles) else theta.shape[0]
        theta, d, acc = theta[:m], d[:m], acc[:m]
        # each record's "parent" in a transition's population (the MFMA KDE
        # pass evaluates the row relative to that particle's term; any index
        # gives the same density): the previous population -- the particle
        # its proposal was resampled from -- and the new one, which holds
        # the accepted records in order, so an accepted record is particle
        # cumsum(acc) - 1 there (rejected: none)
        par_prev = par_cur = None
        if parent is not None:
            par_prev = parent[:m]
            a = acc > 0
            par_cur = torch.where(a, torch.cumsum(a.to(torch.int64), 0) - 1,
                                  torch.full_like(par_prev, -1))
        return DeviceRecords(d, self._log_transition_pd(t - 1, prev_transitions,
                                                        theta, par_prev),
                             self._log_transition_pd(t, self.transitions,
                                                     theta, par_cur), acc)

    def _log_transition_pd(self, t, transitions, theta, parent=None):
        if t == 0:
            # prior density: constant on the (uniform-box) support, where
            # every recorded proposal lies (smc.py:737-749)
            names = self.parameter_priors[0].uniform_box()[0]
            par = Parameter(dict(zip(names, theta[0].cpu().numpy())))
            pd0 = self._create_prior_pdf()(0, par)
            return torch.full((theta.shape[0],), float(np.log(pd0)),
                              dtype=theta.dtype, device=theta.device)
        return transitions[0].logpdf_device(theta, parent)

    def _adapt_population_size(self, t):
        if t == 0:
            return
        w = self.history.get_model_probabilities(self.history.max_t)["p"].values
        self.population_size.update(self.transitions, w, t)

    def _fit_transitions(self, t):
        """smc.py:1047-1061: fit on the previous population (device frame)."""
        if t == 0:
            return
        for m in self.history.alive_models(t - 1):
            particles, w = self.history.get_distribution(m, t - 1)
            self.transitions[m].fit(particles, w)


__all__ = ["ABCSMC", "identity", "fast_random_choice", "Parameter"]
