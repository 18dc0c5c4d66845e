"""The device-aware ``update_field_with_exchange``,
bound into the restated reference Store protocol.

``lens_amd.registry.update_field_with_exchange`` has the reference updater's
signature ``(current_value, new_value, states)`` (vivarium/core/registry.py:
149-183).  A maintainer installs it with one line into the reference's
``updater_registry``; here the same replacement goes into the oracle's
restatement of ``Store.apply_update``'s per-leaf updater protocol
(``oracle.experiment.OracleExperiment``, experiment.py:586-739), which calls
``updater(current, value, states)`` once per agent and molecule.

* CPU: on a numpy field the updater is the reference's arithmetic, bit for bit.
* GPU: a 40-agent colony with 2 device fields (``BatchedDiffusionField`` and
  ``BatchedConvenienceKinetics``, each ``next_update`` a batch of one) run
  through that per-leaf protocol equals the all-oracle run bit for bit, while
  each updater call only queues O(1) host work on the field.
"""

import numpy as np
import pytest

from oracle.experiment import make_update_field_with_exchange as oracle_updater


def _states(loc, n_bins=(13, 9), bounds=(26.0, 9.0), depth=3.0):
    return {'global': {'location': loc}, 'dimensions': {'n_bins': list(n_bins), 'bounds': list(bounds),
                                                        'depth': depth}}


def test_host_field_is_the_reference_arithmetic():
    from lens_amd.registry import update_field_with_exchange
    rng = np.random.default_rng(5)
    f_ref = rng.random((13, 9))
    f_got = f_ref.copy()
    ref = oracle_updater()
    for _ in range(200):
        loc = [float(rng.uniform(-30, 60)), float(rng.uniform(-9, 18))]
        count = int(rng.integers(-10**9, 10**9))
        f_ref = ref(f_ref, count, _states(loc))
        f_got = update_field_with_exchange(f_got, count, _states(loc))
    assert np.array_equal(f_got, f_ref)


def test_avogadro_is_a_parameter():
    from lens_amd.registry import make_update_field_with_exchange
    f = np.zeros((13, 9))
    a = make_update_field_with_exchange(6.022140857e23)(f, 10**12, _states([1.0, 1.0]))
    b = make_update_field_with_exchange(6.02214076e23)(f, 10**12, _states([1.0, 1.0]))
    assert a[0, 1] != b[0, 1]
    assert np.array_equal(a, oracle_updater(6.022140857e23)(f, 10**12, _states([1.0, 1.0])))


# ---------------------------------------------------------------------------
# GPU: the per-leaf protocol with the device-aware updater installed
# ---------------------------------------------------------------------------

NX, NY, N = 24, 20, 40


def _colony(batched, dev):
    from lens_amd import configs
    from lens_amd.process import BatchedConvenienceKinetics, BatchedDiffusionField
    from oracle.experiment import OracleConvenienceKinetics, OracleDiffusionField
    from oracle.kinetics import mmol_to_counts
    cfg = configs.glc_ac_config()
    rng = np.random.default_rng(11)
    locs = [[float(rng.uniform(0, NX)), float(rng.uniform(0, NY))] for _ in range(N)]
    locs[7] = list(locs[3])                      # two agents share a bin: per-bin agent order matters
    locs[19] = list(locs[3])
    glc = configs.gaussian_bump_field((NX, NY))
    env = {'molecules': ['glc__D_e', 'ac_e'], 'n_bins': [NX, NY], 'bounds': [float(NX), float(NY)],
           'depth': 10.0, 'diffusion': 5.0, 'time_step': 2.0,
           'initial_state': {'glc__D_e': glc, 'ac_e': np.zeros((NX, NY))}}
    processes = {'diffusion': BatchedDiffusionField(dict(env, device=dev)) if batched else OracleDiffusionField(env),
                 'agents': {}}
    topology = {'diffusion': {'agents': ('agents',), 'fields': ('fields',), 'dimensions': ('dimensions',)},
                'agents': {}}
    agents = {}
    for a in range(N):
        kin_cfg = dict(cfg, time_step=1.0)
        processes['agents']['a%02d' % a] = {
            'kinetics': BatchedConvenienceKinetics(kin_cfg) if batched else OracleConvenienceKinetics(kin_cfg)}
        topology['agents']['a%02d' % a] = {'kinetics': {
            'internal': ('internal',), 'external': ('boundary', 'external'), 'fluxes': ('fluxes',),
            'fields': ('..', '..', 'fields'), 'dimensions': ('..', '..', 'dimensions'), 'global': ('boundary',)}}
        internal = {k: v * (1 + 0.013 * a) for k, v in cfg['initial_state']['internal'].items()}
        agents['a%02d' % a] = {'internal': internal, 'fluxes': {},
                               'boundary': {'location': locs[a], 'mmol_to_counts': mmol_to_counts(1200.0 + 9 * a),
                                            'external': {'glc__D_e': 0.0, 'ac_e': 0.0}}}
    init = {'agents': agents, 'dimensions': {'bounds': env['bounds'], 'n_bins': env['n_bins'], 'depth': 10.0}}
    return processes, topology, init


def _host(x):
    return x.cpu().numpy() if hasattr(x, 'cpu') else x


def _compare(a, b, path=()):
    if isinstance(b, dict):
        assert isinstance(a, dict) and sorted(a) == sorted(b), path
        for k in b:
            _compare(a[k], b[k], path + (k,))
    else:
        x, y = _host(a), _host(b)
        if isinstance(y, np.ndarray):
            assert np.array_equal(x, y), path
        else:
            assert x == y, (path, x, y)


@pytest.mark.gpu
def test_reference_store_protocol_with_device_exchange_updater():
    torch = pytest.importorskip('torch')
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from lens_amd.registry import DeviceField, update_field_with_exchange
    from oracle.experiment import OracleExperiment
    dev = torch.device('cuda', 0)
    calls = []

    def counted(current, new, states):         # the installed updater, call by call
        out = update_field_with_exchange(current, new, states)
        calls.append((type(current).__name__, out is current, getattr(out, 'pending', None)))
        return out

    p, t, init = _colony(True, dev)
    gpu = OracleExperiment(p, t, init, updater_registry={'update_field_with_exchange': counted})
    p, t, init = _colony(False, dev)
    ref = OracleExperiment(p, t, init)
    assert isinstance(gpu.state['fields']['ac_e'], DeviceField)
    for interval in (1.0, 3.0, 0.5, 4.5):
        calls.clear()
        gpu.update(interval)
        ref.update(interval)
        # one updater call per agent, molecule and kinetics step; none of them touched the
        # lattice (O(1): the field object is returned as it came, with one more queued entry)
        assert calls and all(kind == 'DeviceField' and same for kind, same, _ in calls)
        assert max(pending for _, _, pending in calls) >= N
        _compare(gpu.state['agents'], ref.state['agents'])
        _compare(gpu.state['fields'], ref.state['fields'])
    ac = _host(gpu.state['fields']['ac_e'])
    assert ac.max() > 0 and np.count_nonzero(ac) > N // 2
