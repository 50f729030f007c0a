"""Environment ids, MP configuration merge and flattening to the C-ABI config.

Mirrors (paths relative to /root/reference/fancy_gym):
  _BB_DEFAULTS                 envs/registry.py:62-129
  nested_update                envs/registry.py:264-277   (a dict with a '*_type' key replaces)
  register / upgrade           envs/registry.py:137-220   ('{ns}_{MP}/{name}' ids, registry.py:243)
  bb_env_constructor           envs/registry.py:280-309   (defaults <- MPWrapper.mp_config <- overrides)
  make_bb                      utils/make_env_helpers.py:68-136 (duration, tau, TimeAwareObservation)
  reacher registrations        envs/__init__.py:57-65, 658-666, 669-679, 682-698
  MPWrapper.mp_config          simple_reacher/mp_wrapper.py:10-30, hole_reacher/mp_wrapper.py:10-32,
                               viapoint_reacher/mp_wrapper.py:10-25
Third-party defaults restated from mp_pytorch<=0.1.3 [EXT-M] (not in the container).
"""
import copy
import math
from collections.abc import Mapping

import numpy as np

from . import _lib

_BB_DEFAULTS = {
    'ProMP': {
        'wrappers': [],
        'trajectory_generator_kwargs': {'trajectory_generator_type': 'promp'},
        'phase_generator_kwargs': {'phase_generator_type': 'linear'},
        'controller_kwargs': {'controller_type': 'motor', 'p_gains': 1.0, 'd_gains': 0.1},
        'basis_generator_kwargs': {'basis_generator_type': 'zero_rbf', 'num_basis': 5,
                                   'num_basis_zero_start': 1, 'basis_bandwidth_factor': 3.0},
        'black_box_kwargs': {},
    },
    'DMP': {
        'wrappers': [],
        'trajectory_generator_kwargs': {'trajectory_generator_type': 'dmp'},
        'phase_generator_kwargs': {'phase_generator_type': 'exp'},
        'controller_kwargs': {'controller_type': 'motor', 'p_gains': 1.0, 'd_gains': 0.1},
        'basis_generator_kwargs': {'basis_generator_type': 'rbf', 'num_basis': 5},
        'black_box_kwargs': {},
    },
    'ProDMP': {
        'wrappers': [],
        'trajectory_generator_kwargs': {'trajectory_generator_type': 'prodmp', 'duration': 2.0,
                                        'weights_scale': 1.0},
        'phase_generator_kwargs': {'phase_generator_type': 'exp', 'tau': 1.5},
        'controller_kwargs': {'controller_type': 'motor', 'p_gains': 1.0, 'd_gains': 0.1},
        'basis_generator_kwargs': {'basis_generator_type': 'prodmp', 'alpha': 10, 'num_basis': 5},
        'black_box_kwargs': {},
    },
}
KNOWN_MPS = list(_BB_DEFAULTS.keys())

# mp_pytorch<=0.1.3 constructor defaults [EXT-M]
_MP_PYTORCH_DEFAULTS = dict(alpha_phase=3.0, delay=0.0, basis_bandwidth_factor=3.0, num_basis_zero_start=2,
                            num_basis_zero_goal=0, dmp_alpha=25.0, prodmp_alpha=25.0,
                            pre_compute_length_factor=6.0, weights_scale=1.0, goal_scale=1.0)


class EnvSpec:
    """A registered step-based env (what gym.make('fancy/<Name>-v0') builds)."""

    def __init__(self, id, kind, kwargs, max_episode_steps, mp_config, traj_validity=None):
        self.id = id
        self.traj_validity = traj_validity    # TrajValidity (the MPWrapper's validity hooks) or None
        self.kind = kind                      # 'simple' (torque) | 'hole' | 'via' (direct velocity)
        self.kwargs = dict(kwargs)
        self.max_episode_steps = max_episode_steps
        self.mp_config = mp_config


_SIMPLE_MP_CONFIG = {   # simple_reacher/mp_wrapper.py:10-30
    'ProMP': {'controller_kwargs': {'p_gains': 0.6, 'd_gains': 0.075}},
    'DMP': {'controller_kwargs': {'p_gains': 0.6, 'd_gains': 0.075},
            'trajectory_generator_kwargs': {'weights_scale': 50},
            'phase_generator_kwargs': {'alpha_phase': 2}},
    'ProDMP': {},
}
_HOLE_MP_CONFIG = {     # hole_reacher/mp_wrapper.py:10-32
    'ProMP': {'controller_kwargs': {'controller_type': 'velocity'},
              'trajectory_generator_kwargs': {'weights_scale': 2}},
    'DMP': {'controller_kwargs': {'controller_type': 'velocity'},
            'trajectory_generator_kwargs': {'weights_scale': 500},
            'phase_generator_kwargs': {'alpha_phase': 2.5}},
    'ProDMP': {},
}

_VIA_MP_CONFIG = {      # viapoint_reacher/mp_wrapper.py:10-25
    'ProMP': {'controller_kwargs': {'controller_type': 'velocity'}},
    'DMP': {'controller_kwargs': {'controller_type': 'velocity'},
            'trajectory_generator_kwargs': {'weights_scale': 50},
            'phase_generator_kwargs': {'alpha_phase': 2}},
    'ProDMP': {},
}

ENV_SPECS = {}
ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS = {k: [] for k in KNOWN_MPS + ['all']}
MOVEMENT_PRIMITIVE_ENVIRONMENTS_FOR_NS = {}


def nested_update(base, update):
    """registry.py:264-277: a mapping containing any '*_type' key replaces the sub-dict."""
    if any(item.endswith('_type') for item in update):
        return update
    for k, v in update.items():
        base[k] = nested_update(base.get(k, {}), v) if isinstance(v, Mapping) else v
    return base


def register(id, kind, kwargs, max_episode_steps=200, mp_config=None, add_mp_types=KNOWN_MPS,
             mp_config_override=None, traj_validity=None):
    """Register a step-based reacher id and its '{ns}_{MP}/{name}' black-box ids (registry.py:137-183).
    traj_validity: TrajValidity, the variant's MPWrapper validity hooks (default: every plan valid)."""
    spec = EnvSpec(id, kind, kwargs, max_episode_steps, mp_config or {}, traj_validity)
    ENV_SPECS[id] = spec
    upgrade(id, add_mp_types=add_mp_types, mp_config_override=mp_config_override)
    return spec


def upgrade(id, add_mp_types=KNOWN_MPS, base_id=None, mp_config_override=None):
    """registry.py:186-261."""
    base_id = base_id or id
    for mp_type in add_mp_types:
        assert mp_type in KNOWN_MPS, 'Unknown mp_type'
        parts = id.split('/')
        if len(parts) == 1:
            ns, name = 'gym', parts[0]
        elif len(parts) == 2:
            ns, name = parts
        else:
            raise ValueError('env id can not contain multiple "/".')
        p2 = name.split('-')
        assert len(p2) >= 2 and p2[-1].startswith('v'), 'Malformed env id, must end in -v{int}.'
        fancy_id = f'{ns}_{mp_type}/{name}'
        assert fancy_id not in ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS[mp_type], \
            f'The environment {id} is already registered for {mp_type}.'
        _BB_IDS[fancy_id] = (base_id, mp_type, copy.deepcopy((mp_config_override or {}).get(mp_type, {})))
        ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS[mp_type].append(fancy_id)
        ALL_MOVEMENT_PRIMITIVE_ENVIRONMENTS['all'].append(fancy_id)
        d = MOVEMENT_PRIMITIVE_ENVIRONMENTS_FOR_NS.setdefault(ns, {k: [] for k in KNOWN_MPS + ['all']})
        d[mp_type].append(fancy_id)
        d['all'].append(fancy_id)


_BB_IDS = {}

# envs/__init__.py:57-65, 658-666, 682-698
register('fancy/SimpleReacher-v0', 'simple', {'n_links': 2}, 200, _SIMPLE_MP_CONFIG)
register('fancy/LongSimpleReacher-v0', 'simple', {'n_links': 5}, 200, _SIMPLE_MP_CONFIG)
register('fancy/HoleReacher-v0', 'hole', {'n_links': 5, 'random_start': True, 'allow_self_collision': False,
                                          'allow_wall_collision': False, 'hole_width': None,
                                          'hole_depth': 1, 'hole_x': None, 'collision_penalty': 100},
         200, _HOLE_MP_CONFIG)
register('fancy/ViaPointReacher-v0', 'via', {'n_links': 5, 'allow_self_collision': False, 'collision_penalty': 1000},
         200, _VIA_MP_CONFIG)


# --------------------------------------------------------------------------- replanning schedules
# ``replanning_schedule(pos, vel, obs, action, t) -> bool`` (black_box_wrapper.py:233) runs on the
# device as a small clause program (include/fgx.h FGX_SCHED_*): the OR of up to four clauses.
# Each class below is also a plain callable with the reference's signature, so the same object
# can be handed to the reference's BlackBoxWrapper.
class _Clause:
    def clauses(self):
        return [self]

    def __or__(self, other):
        return ReplanAny(self, other)


class ReplanEvery(_Clause):
    """t % period == 0 (example_replanning_envs.py:37-39, the reference's mp_wrapper schedules)."""

    def __init__(self, period):
        if int(period) <= 0:
            raise ValueError("period must be positive")
        self.period = int(period)

    def __call__(self, pos, vel, obs, action, t):
        return t % self.period == 0

    def batch(self, obs, t):
        return np.asarray(t) % self.period == 0

    def encode(self):
        return (_lib.SCHED_EVERY, self.period, 0, 0, 0.0, 1.0)


class ReplanAt(_Clause):
    """t == step."""

    def __init__(self, step):
        self.step = int(step)

    def __call__(self, pos, vel, obs, action, t):
        return t == self.step

    def batch(self, obs, t):
        return np.asarray(t) == self.step

    def encode(self):
        return (_lib.SCHED_AT, self.step, 0, 0, 0.0, 1.0)


class ReplanNormPeriod(_Clause):
    """t % max(int(np.linalg.norm(obs[i0:i1]) ** 2 * mul / div), 1) == 0 — the state-dependent
    period of crowd_navigation/utils.py:9-10 (obs is the time-aware observation)."""

    def __init__(self, i0, i1, mul, div=1.0):
        self.i0, self.i1, self.mul, self.div = int(i0), int(i1), float(mul), float(div)
        if not (0 <= self.i0 < self.i1 <= self.i0 + 8) or self.div == 0.0:
            raise ValueError("need 0 <= i0 < i1 <= i0 + 8 and div != 0")

    def _period(self, o):
        return max(int(np.linalg.norm(o[self.i0:self.i1]) ** 2 * self.mul / self.div), 1)

    def __call__(self, pos, vel, obs, action, t):
        return t % self._period(np.asarray(obs)) == 0

    def batch(self, obs, t):
        return np.array([int(ti) % self._period(o) == 0 for o, ti in zip(obs, np.asarray(t))], bool)

    def encode(self):
        return (_lib.SCHED_NORM_PERIOD, 0, self.i0, self.i1, self.mul, self.div)


class ReplanAny(_Clause):
    """OR of clauses (at most four on the device)."""

    def __init__(self, *clauses):
        flat = []
        for c in clauses:
            flat += c.clauses()
        if not 1 <= len(flat) <= 4:
            raise ValueError("a device schedule has 1..4 clauses")
        self._clauses = flat

    def clauses(self):
        return list(self._clauses)

    def __call__(self, pos, vel, obs, action, t):
        return any(c(pos, vel, obs, action, t) for c in self._clauses)

    def batch(self, obs, t):
        out = np.zeros(len(np.asarray(t)), bool)
        for c in self._clauses:
            out |= c.batch(obs, t)
        return out


# crowd_navigation/utils.py:9-10 ``replan_close``
REPLAN_CLOSE = ReplanAny(ReplanEvery(10), ReplanNormPeriod(0, 2, 10, 4))


def _compile_schedule(schedule, max_steps):
    """replanning_schedule -> device clause list.  Clause objects compile directly; a plain
    callable is probed: it must be a pure function of t, of the form t % k == 0 or firing at
    <= 4 fixed steps.  State-dependent lambdas must be written with ReplanNormPeriod."""
    if schedule is None:
        return []
    if isinstance(schedule, _Clause):
        return [c.encode() for c in schedule.clauses()]
    if isinstance(schedule, (int, np.integer)):
        return [ReplanEvery(int(schedule)).encode()]
    if not callable(schedule):
        raise ValueError("replanning_schedule must be callable or an int period")
    dummy = np.zeros(1)
    try:
        hits = [t for t in range(1, max_steps + 1) if bool(schedule(dummy, dummy, dummy, dummy, t))]
        probe = [t for t in range(1, max_steps + 1)
                 if bool(schedule(dummy + 1.0, dummy - 1.0, dummy + 2.0, dummy + 3.0, t))]
    except Exception as e:   # state-dependent schedules (crowd_navigation/utils.py:9-10)
        raise NotImplementedError(f"replanning_schedule is not a pure function of t ({e}); "
                                  "express it with fgx.ReplanNormPeriod / ReplanAny")
    if hits != probe:
        raise NotImplementedError("state-dependent replanning_schedule: express it with "
                                  "fgx.ReplanNormPeriod / ReplanAny")
    if not hits:
        return []
    k = hits[0]
    if hits == list(range(k, max_steps + 1, k)):
        return [ReplanEvery(k).encode()]
    if len(hits) <= 4:
        return [ReplanAt(t).encode() for t in hits]
    raise NotImplementedError("only t % k == 0, <= 4 fixed steps or fgx.Replan* clause schedules run on the device")


def _schedule_period(schedule, max_steps):
    """Period of a pure t % k == 0 schedule (0: none); raises for anything else."""
    cl = _compile_schedule(schedule, max_steps)
    if not cl:
        return 0
    if len(cl) == 1 and cl[0][0] == _lib.SCHED_EVERY:
        return cl[0][1]
    raise NotImplementedError("not a t % k == 0 schedule")


# --------------------------------------------------------------------------- trajectory validity
class TrajValidity:
    """The env-side validity hooks of a black-box env, run on the device (include/fgx.h FGX_VALID_*):
    RawInterfaceWrapper.preprocessing_and_validity_callback / invalid_traj_callback
    (raw_interface_wrapper.py:55-72,103-121, called at black_box_wrapper.py:178-197).  The registered
    reachers keep the reference's identity default (every plan valid); a registered variant or a
    make() call passes ``traj_validity=TrajValidity(...)`` for the checks the reference's overriding
    envs make (table_tennis_env.py:304-309):

      tau=(lo, hi)        raw learned tau action[0] inside [lo, hi]          (needs learn_tau)
      delay=(lo, hi)      raw learned delay action[learn_tau] inside [lo, hi] (needs learn_delay)
      pos_low / pos_high  per-joint bounds on the desired positions of the whole plan

    An invalid plan yields the artificial transition (no env step, trajectory_length 0):
    return ``invalid_return``, ``terminated`` / ``truncated`` as given (reference default: True /
    False), observation zeros (``obs='zeros'``, np.zeros) or the env's current one
    (``obs='current'``).  ``__call__`` is the host predicate with the reference's signature.

    Comparison semantics follow numpy >= 2 (NEP 50), the numpy of this image: the raw float32 action
    entry is compared with a Python-float bound in float32 (the bound rounded to f32 first); under
    numpy 1.x value-based casting the same comparison ran in float64, so an action within one f32 ulp
    of a bound that is not an f32 value can be classed differently there.  Pinned by
    tests/test_host_cpu.py::test_validity_bound_semantics_follow_nep50 (host) and
    tests/test_gpu_validity.py::test_tau_bound_one_ulp (device)."""

    def __init__(self, tau=None, delay=None, pos_low=None, pos_high=None, invalid_return=0.0,
                 terminated=True, truncated=False, obs='zeros'):
        if obs not in ('zeros', 'current'):
            raise ValueError("obs must be 'zeros' or 'current'")
        if (pos_low is None) != (pos_high is None):
            raise ValueError("pos_low and pos_high go together")
        self.tau = None if tau is None else (float(tau[0]), float(tau[1]))
        self.delay = None if delay is None else (float(delay[0]), float(delay[1]))
        self.pos_low = None if pos_low is None else np.asarray(pos_low, np.float64).reshape(-1)
        self.pos_high = None if pos_high is None else np.asarray(pos_high, np.float64).reshape(-1)
        self.invalid_return = float(invalid_return)
        self.terminated, self.truncated, self.obs = bool(terminated), bool(truncated), obs

    def __call__(self, action, pos_traj, vel_traj, tau_bound=None, delay_bound=None, learn_tau=True):
        """(valid, pos_traj, vel_traj) for one env, as preprocessing_and_validity_callback."""
        a = np.asarray(action, np.float32)
        if self.tau is not None and (a[0] > self.tau[1] or a[0] < self.tau[0]):
            return False, pos_traj, vel_traj
        i = 1 if learn_tau else 0
        if self.delay is not None and (a[i] > self.delay[1] or a[i] < self.delay[0]):
            return False, pos_traj, vel_traj
        if self.pos_low is not None and (np.any(pos_traj > self.pos_high) or np.any(pos_traj < self.pos_low)):
            return False, pos_traj, vel_traj
        return True, pos_traj, vel_traj

    def encode(self, c, n_links):
        flags = 0
        if self.tau is not None:
            if not c.learn_tau:
                raise ValueError("TrajValidity(tau=...) needs learn_tau")
            flags |= _lib.VALID_TAU
            c.valid_tau_lo, c.valid_tau_hi = self.tau
        if self.delay is not None:
            if not c.learn_delay:
                raise ValueError("TrajValidity(delay=...) needs learn_delay")
            flags |= _lib.VALID_DELAY
            c.valid_delay_lo, c.valid_delay_hi = self.delay
        if self.pos_low is not None:
            lo = np.broadcast_to(self.pos_low, (n_links,)) if self.pos_low.size in (1, n_links) else self.pos_low
            hi = np.broadcast_to(self.pos_high, (n_links,)) if self.pos_high.size in (1, n_links) else self.pos_high
            if lo.shape != (n_links,) or hi.shape != (n_links,):
                raise ValueError(f"pos_low / pos_high need {n_links} entries")
            flags |= _lib.VALID_POS
            for k in range(n_links):
                c.valid_pos_lo[k], c.valid_pos_hi[k] = float(lo[k]), float(hi[k])
        c.valid_flags = flags
        c.invalid_reward = self.invalid_return
        c.invalid_terminated, c.invalid_truncated = int(self.terminated), int(self.truncated)
        c.invalid_obs = _lib.INVALID_OBS_CURRENT if self.obs == 'current' else _lib.INVALID_OBS_ZEROS


# --------------------------------------------------------------------------- resolution
def parse_id(env_id):
    ns_mp, _, name = env_id.partition('/')
    if env_id in ENV_SPECS:
        return env_id, None, {}
    if env_id not in _BB_IDS:
        raise ValueError(f"unknown env id {env_id!r}; known: {sorted(list(ENV_SPECS) + list(_BB_IDS))}")
    base_id, mp_type, reg_override = _BB_IDS[env_id]
    return base_id, mp_type, reg_override


def resolve(env_id, mp_config_override=None, **env_kwargs):
    """id (+ overrides) -> (fgx_config, meta) exactly as bb_env_constructor + make_bb resolve it."""
    base_id, mp_type, reg_override = parse_id(env_id)
    spec = ENV_SPECS[base_id]
    kw = dict(spec.kwargs)
    kw.update(env_kwargs)
    validity = kw.pop('traj_validity', spec.traj_validity)
    if validity is not None and not isinstance(validity, TrajValidity):
        raise ValueError("traj_validity must be a fgx.TrajValidity")
    c = _lib.FgxConfig()
    c.abi_version = _lib.FGX_ABI_VERSION
    n = int(kw['n_links'])
    if not 1 <= n <= 8:   # the engine's register-resident joint arrays (include/fgx.h n_links 1..8)
        raise ValueError(f"n_links must be in 1..8, got {n}")
    if spec.kind == 'hole' and n == 1 and not kw.get('allow_wall_collision', False):
        # the reference's wall check indexes np.squeeze(line_points) as [link, point, xy]; one link
        # squeezes to [point, xy] and its first step raises (hole_reacher.py:126-148)
        raise IndexError("too many indices for array: HoleReacher with n_links=1 cannot run its wall check "
                         "(hole_reacher.py:143); pass allow_wall_collision=True")
    c.n_links = n
    c.env_kind = {'simple': _lib.ENV_SIMPLE, 'hole': _lib.ENV_HOLE, 'via': _lib.ENV_VIA}[spec.kind]
    # constructor defaults: SimpleReacherEnv random_start=True; HoleReacherEnv / ViaPointReacherEnv False
    rs_default = spec.kind == 'simple'
    c.random_start = int(bool(kw.get('random_start', rs_default)))
    c.allow_self_collision = int(bool(kw.get('allow_self_collision', False)))
    c.allow_wall_collision = int(bool(kw.get('allow_wall_collision', False)))
    c.dt = 0.01                                                # base_reacher.py:21
    c.max_episode_steps = int(spec.max_episode_steps)
    nan = float('nan')
    c.hole_width = c.hole_depth = c.hole_x = nan
    c.via_x = c.via_y = c.target_x = c.target_y = nan
    c.rew_fct = _lib.REW_SIMPLE
    if spec.kind == 'hole':
        c.hole_width = nan if kw.get('hole_width', 1.0) is None else float(kw.get('hole_width', 1.0))
        c.hole_depth = nan if kw.get('hole_depth') is None else float(kw['hole_depth'])
        c.hole_x = nan if kw.get('hole_x') is None else float(kw['hole_x'])
        c.collision_penalty = float(kw.get('collision_penalty', 1000))
        bound = float(np.float32(2 * np.pi))                   # Box(float32) bounds, base_reacher_direct.py:16-18
        rew = kw.get('rew_fct', 'simple')                      # hole_reacher.py:48-58
        if rew not in ('simple', 'vel_acc', 'unbounded'):
            raise ValueError("Unknown reward function {}".format(rew))
        c.rew_fct = {'simple': _lib.REW_SIMPLE, 'vel_acc': _lib.REW_VEL_ACC, 'unbounded': _lib.REW_UNBOUNDED}[rew]
    elif spec.kind == 'via':
        c.collision_penalty = float(kw.get('collision_penalty', 1000))
        bound = float(np.float32(2 * np.pi))
        for key, (fx, fy) in (('via_target', ('via_x', 'via_y')), ('target', ('target_x', 'target_y'))):
            v = kw.get(key)
            if v is not None:
                v = np.asarray(v, dtype=np.float64).reshape(-1)
                if v.shape != (2,):
                    raise ValueError(f"{key} must be an (x, y) pair")
                setattr(c, fx, float(v[0]))
                setattr(c, fy, float(v[1]))
    else:
        bound = 1000.0                                          # base_reacher_torque.py:16-18
        if kw.get('target') is not None:                        # simple_reacher.py:19,93-94
            v = np.asarray(kw['target'], dtype=np.float64).reshape(-1)
            if v.shape != (2,):
                raise ValueError("target must be an (x, y) pair")
            c.target_x, c.target_y = float(v[0]), float(v[1])
    c.act_low, c.act_high = -bound, bound
    # verbose: BlackBoxWrapper.step(action, verbose=2) — the reference's step always assembles the
    # verbose-2 info (black_box_wrapper.py:170,185,244-249) whatever black_box_kwargs['verbose'] is
    meta = dict(env_id=env_id, base_id=base_id, mp_type=mp_type, kind=spec.kind, n_links=n,
                reward_aggregation='sum', verbose=2)
    if mp_type is None:                                          # step-based env
        c.mp_kind = _lib.MP_NONE
        c.T = 1
        c.return_context = 0
        return c, meta

    # ---- bb_env_constructor (registry.py:280-309)
    mp_config = spec.mp_config
    active = copy.deepcopy(mp_config.get(mp_type, {}))
    inherit = active.pop('inherit_defaults', mp_config.get('inherit_defaults', True))
    config = copy.deepcopy(_BB_DEFAULTS[mp_type]) if inherit else {}
    config = nested_update(config, active)
    config = nested_update(config, copy.deepcopy(reg_override))
    config = nested_update(config, copy.deepcopy(mp_config_override or {}))
    wrappers = config.pop('wrappers', [])
    tg = config.pop('trajectory_generator_kwargs', {})
    bb = config.pop('black_box_kwargs', {})
    ctrl = config.pop('controller_kwargs', {})
    ph = config.pop('phase_generator_kwargs', {})
    bs = config.pop('basis_generator_kwargs', {})

    # ---- make_bb (make_env_helpers.py:68-136)
    if bb.get('learn_sub_trajectories') and bb.get('replanning_schedule'):
        raise ValueError('Cannot used sub-trajectory learning and replanning together.')
    learn_sub = bool(bb.get('learn_sub_trajectories'))
    learn_tau = bool(ph.get('learn_tau', False))
    learn_delay = bool(ph.get('learn_delay', False))
    if bb.get('learn_sub_trajectories') is not None:   # make_env_helpers.py:115-116 ("is not None")
        learn_tau = True
    duration = bb.get('duration')
    if duration is None:
        duration = c.max_episode_steps * c.dt
    if tg.get('duration') is not None and bb.get('time_limit') is not None:
        assert tg['duration'] == bb['time_limit']
    tau = ph.get('tau', duration)
    if tau is None:
        tau = duration
    action_dim = int(tg.get('action_dim', n))
    if action_dim != n:
        raise ValueError("action_dim must equal n_links for the reacher envs")
    sched = _compile_schedule(bb.get('replanning_schedule'), c.max_episode_steps)
    period = sched[0][1] if (len(sched) == 1 and sched[0][0] == _lib.SCHED_EVERY) else 0
    do_replanning = len(sched) > 0
    time_aware = (do_replanning or learn_sub or
                  any(getattr(w, '__name__', '') == 'TimeAwareObservation' for w in wrappers))

    tg_type = tg.get('trajectory_generator_type', '').lower()
    ph_type = ph.get('phase_generator_type', '').lower()
    bs_type = bs.get('basis_generator_type', '').lower()
    ct_type = ctrl.get('controller_type', '').lower()
    c.mp_kind = {'promp': _lib.MP_PROMP, 'dmp': _lib.MP_DMP, 'prodmp': _lib.MP_PRODMP}.get(tg_type, -1)
    if c.mp_kind < 0:
        raise ValueError(f"Specified movement primitive type {tg_type} not supported")
    c.phase_kind = {'linear': _lib.PHASE_LINEAR, 'exp': _lib.PHASE_EXP}.get(ph_type, -1)
    if c.phase_kind < 0:
        raise ValueError(f"Specified phase generator type {ph_type} not supported")
    if bs_type not in ('rbf', 'zero_rbf', 'prodmp'):
        raise ValueError(f"Specified basis generator type {bs_type} not supported")
    if bs_type == 'prodmp' and ph_type != 'exp':
        raise AssertionError("ProDMP basis needs the exp phase generator")
    if (tg_type == 'prodmp') != (bs_type == 'prodmp'):
        raise AssertionError("prodmp trajectory generator needs the prodmp basis generator")
    c.ctrl_kind = {'motor': _lib.CTRL_PD, 'velocity': _lib.CTRL_VEL, 'position': _lib.CTRL_POS}.get(ct_type, -1)
    if c.ctrl_kind < 0:
        raise ValueError(f"Specified controller type {ct_type} not supported")
    D = _MP_PYTORCH_DEFAULTS
    c.n_basis = int(bs.get('num_basis', 10))
    c.zero_start = int(bs.get('num_basis_zero_start', D['num_basis_zero_start'])) if bs_type == 'zero_rbf' else 0
    c.zero_goal = int(bs.get('num_basis_zero_goal', D['num_basis_zero_goal'])) if bs_type == 'zero_rbf' else 0
    # num_basis_outside (mp_pytorch NormalizedRBF / ProDMP basis generators): centres beyond the
    # phase's [0, 1]; the zero-padding generator takes no such argument
    c.num_basis_outside = int(bs.get('num_basis_outside', 0))
    if c.num_basis_outside and bs_type == 'zero_rbf':
        raise TypeError("ZeroPaddingNormalizedRBFBasisGenerator got an unexpected keyword argument "
                        "'num_basis_outside'")
    if c.num_basis_outside < 0 or c.n_basis - 2 * c.num_basis_outside - 1 < 1:
        raise ValueError("num_basis_outside must satisfy 0 <= o and num_basis - 2 o > 1")
    c.bandwidth = float(bs.get('basis_bandwidth_factor', D['basis_bandwidth_factor']))
    c.tau = float(tau)
    c.delay = float(ph.get('delay', D['delay']))
    c.alpha_phase = float(ph.get('alpha_phase', D['alpha_phase']))
    c.weights_scale = float(tg.get('weights_scale', D['weights_scale']))
    c.goal_scale = float(tg.get('goal_scale', D['goal_scale']))
    if tg_type == 'prodmp':
        c.alpha = float(bs.get('alpha', D['prodmp_alpha']))
        c.pc_length = float(bs.get('pre_compute_length_factor', D['pre_compute_length_factor']))
        # the ProDMP basis generator's own dt (its precompute grid, basis_generator_factory.py:8-23);
        # rows are looked up at the rounded grid index of each env step (fgx_tables.h)
        c.basis_dt = float(bs.get('dt', c.dt))
        if not (c.basis_dt > 0.0):
            raise ValueError("basis generator dt must be positive")
    else:
        if 'dt' in bs:   # NormalizedRBF / ZeroPadding generators take no dt (mp_pytorch constructors)
            raise TypeError(f"{bs_type} basis generator got an unexpected keyword argument 'dt'")
        c.alpha = float(tg.get('alpha', D['dmp_alpha']))
        c.pc_length = D['pre_compute_length_factor']
    # PDController(p_gains, d_gains) (pd_controller.py:16-29): scalars or one gain per joint
    pg = np.asarray(ctrl.get('p_gains', 1), dtype=np.float64)
    dg = np.asarray(ctrl.get('d_gains', 0.5), dtype=np.float64)
    if pg.ndim == 0 and dg.ndim == 0:
        c.p_gain, c.d_gain, c.n_gains = float(pg), float(dg), 0
    else:
        pg, dg = np.broadcast_to(pg.reshape(-1), (n,)) if pg.size in (1, n) else pg, \
            np.broadcast_to(dg.reshape(-1), (n,)) if dg.size in (1, n) else dg
        if pg.shape != (n,) or dg.shape != (n,):
            raise ValueError(f"operands could not be broadcast: gains {pg.shape}/{dg.shape} for {n} joints")
        c.n_gains = n
        c.p_gain, c.d_gain = float(pg[0]), float(dg[0])
        for k in range(n):
            c.p_gains[k], c.d_gains[k] = float(pg[k]), float(dg[k])
    c.T = int(round(duration / c.dt))
    c.duration = float(duration)
    c.replan_period = int(period)
    c.sched_n = len(sched)
    for j, (kind, k, i0, i1, mul, div) in enumerate(sched):
        c.sched_kind[j], c.sched_k[j], c.sched_i0[j], c.sched_i1[j] = kind, k, i0, i1
        c.sched_mul[j], c.sched_div[j] = mul, div
    mpt = bb.get('max_planning_times', math.inf)
    c.max_planning_times = 0 if mpt is None or mpt == math.inf else int(mpt)
    c.condition_on_desired = int(bool(bb.get('condition_on_desired', False)))
    c.time_aware = int(time_aware)
    c.return_context = int(not (do_replanning or learn_sub))
    # learned phase parameters (make_env_helpers.py:115-126): bounds two env steps .. duration
    c.learn_tau, c.learn_delay, c.learn_sub_trajectories = int(learn_tau), int(learn_delay), int(learn_sub)
    tb = ph.get('tau_bound') or [c.dt * 2, duration]
    db = ph.get('delay_bound') or [0, duration - c.dt * 2]
    c.tau_bound_lo, c.tau_bound_hi = float(tb[0]), float(tb[1])
    c.delay_bound_lo, c.delay_bound_hi = float(db[0]), float(db[1])
    # reward_aggregation (black_box_wrapper.py:252): np.sum / np.mean run in the episode kernel
    # (numpy's pairwise sum); any other callable is applied to each env's rewards[:t+1]
    agg = bb.get('reward_aggregation', np.sum)
    if agg is np.sum:
        meta['reward_aggregation'] = 'sum'
    elif agg is np.mean:
        meta['reward_aggregation'] = 'mean'
    elif callable(agg):
        meta['reward_aggregation'] = agg
    else:
        raise ValueError("reward_aggregation must be callable")
    meta['n_params'] = n * c.n_basis + (0 if tg_type == 'promp' else n) + int(learn_tau) + int(learn_delay)
    if validity is not None:
        validity.encode(c, n)
    meta['traj_validity'] = validity
    return c, meta
