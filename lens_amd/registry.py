"""Device-aware updaters for the reference's ``updater_registry``.

The reference applies every agent's exchange with the environment through the
updater ``update_field_with_exchange(current_value, new_value, states)``
(vivarium/core/registry.py:149-183), called once per agent and molecule by
``Store.apply_update`` (vivarium/core/experiment.py:715-739).  Each call
allocates ``np.zeros(n_bins)``, puts ``count / (bin_volume * N_A)`` mM into
the agent's bin and returns ``field + delta``: O(lattice) per agent (55 ms
per agent at 4096^2).

:func:`update_field_with_exchange` below has the same signature and result.
On a numpy field it is the reference's arithmetic.  On a field that lives on
the GPU -- a :class:`DeviceField`, or a bare torch device tensor, which it
wraps -- a call costs O(1) host work: the agent's (bin, count) is appended to
the field's queue, and the queue is scattered the first time anything reads
the field, by one agent-ordered ``vk_exchange_sorted`` launch.  That kernel
adds a bin's agents in queue (= call) order, ``((f + c1) + c2) + ...``, which
is what the reference's one-agent-at-a-time ``field + delta`` computes at that
bin (``delta = 0 + c`` is exact), so the field is bit-identical.

Binding it into the reference is one line (the Registry refuses to
re-register a name, so the entry is replaced)::

    from vivarium.core.registry import updater_registry
    from lens_amd.registry import update_field_with_exchange
    updater_registry.registry['update_field_with_exchange'] = update_field_with_exchange

Every reader of a :class:`DeviceField` flushes first: ``.tensor``, numpy
conversion (``np.asarray``, emitters), ``.cpu()``, indexing
(NonSpatialEnvironment's ``field[0][0]``) and ``+`` (the accumulate updater
that applies DiffusionField's delta: a new field, as the reference's
``current + delta`` is a new array).  A ``set`` update replaces the object, and
with it the queued additions -- as the reference's ``set`` discards them.
Signed zeros are the one difference: the reference's ``field + zeros`` turns a
-0.0 bin into +0.0, the device field keeps it (equal under ``==``).
"""

from __future__ import annotations

import math

import numpy as np

from lens_amd.lattice import N_A_LEGACY

__all__ = ['DeviceField', 'update_field_with_exchange', 'make_update_field_with_exchange', 'as_device_tensor',
           'flush_all']


def _bin_site(location, n_bins, bounds):
    """get_bin_site (vivarium/library/lattice_utils.py:18-40): floor(loc*n/bound) % n."""
    i = int(math.floor(location[0] * n_bins[0] / bounds[0])) % int(n_bins[0])
    j = int(math.floor(location[1] * n_bins[1] / bounds[1])) % int(n_bins[1])
    return i, j


def _bin_volume(n_bins, bounds, depth):
    """get_bin_volume (lattice_utils.py:43-58), litres."""
    return (depth * bounds[0] * bounds[1]) * 1e-15 / (n_bins[0] * n_bins[1])


class DeviceField:
    """One diffusion_field plane on the GPU as a Store value, with a queue of
    exchange additions that lands before anything reads the plane."""

    __array_ufunc__ = None          # numpy defers to __radd__ (ndarray + DeviceField)

    def __init__(self, tensor):
        import torch
        if not (isinstance(tensor, torch.Tensor) and tensor.is_cuda and tensor.dim() == 2
                and tensor.dtype == torch.float64):
            raise TypeError('DeviceField wraps a 2-D float64 device tensor')
        self._t = tensor.contiguous()
        self._bins = []             # linear bin per queued call, in call order
        self._counts = []
        self._bva = None            # bin_volume * N_A of the queued calls

    # -- the exchange queue -----------------------------------------------------
    def queue_exchange(self, bin_lin: int, count: int, binvol_avogadro: float):
        if self._bva is not None and binvol_avogadro != self._bva:
            self.flush()            # another bin volume: land the earlier calls first
        self._bva = binvol_avogadro
        self._bins.append(bin_lin)
        self._counts.append(count)

    def queue_exchange_many(self, bins, counts, binvol_avogadro: float):
        """:meth:`queue_exchange` for several calls at once, in list order."""
        if self._bva is not None and binvol_avogadro != self._bva:
            self.flush()
        self._bva = binvol_avogadro
        self._bins.extend(bins)
        self._counts.extend(np.asarray(counts, dtype=np.int64).tolist())

    @property
    def pending(self) -> int:
        return len(self._bins)

    def flush(self):
        """Scatter the queued calls: one ``vk_exchange_sorted`` launch, agent
        (call) order within every bin.  In place on the plane."""
        if not self._bins:
            return self
        import torch
        from lens_amd import native
        from lens_amd.lattice import occupancy
        dev = self._t.device
        k = len(self._bins)
        bins = torch.tensor(self._bins, dtype=torch.int32).to(dev, non_blocking=True)
        counts = torch.tensor(self._counts, dtype=torch.int64).reshape(1, k).to(dev, non_blocking=True)
        bva = self._bva
        self._bins, self._counts, self._bva = [], [], None
        occ_bin, occ_ptr, occ_agent = occupancy(bins, k)
        zero = torch.zeros(1, dtype=torch.int32, device=dev)
        native.load()
        with torch.cuda.device(dev):
            native.check(native._lib.vk_exchange_sorted(
                native.ptr(self._t), self._t.numel(), native.ptr(occ_bin), native.ptr(occ_ptr),
                native.ptr(occ_agent), int(occ_bin.numel()), native.ptr(counts), k, native.ptr(zero),
                native.ptr(zero), 1, bva, native.stream_handle()), 'vk_exchange_sorted')
        return self

    # -- readers (each lands the queue first) ----------------------------------
    @property
    def tensor(self):
        """The plane (a [nx, ny] float64 device tensor), queue landed."""
        self.flush()
        return self._t

    @property
    def shape(self):
        return tuple(self._t.shape)

    @property
    def dtype(self):
        return self._t.dtype

    @property
    def device(self):
        return self._t.device

    @property
    def is_cuda(self):
        return True

    def cpu(self):
        return self.tensor.cpu()

    def numpy(self):
        return self.cpu().numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)

    def __getitem__(self, idx):
        return self.tensor[idx]

    def __add__(self, other):
        """The accumulate updater's ``current + delta``: a new field."""
        return DeviceField(self.tensor + as_device_tensor(other, self._t.device))

    def __radd__(self, other):
        return DeviceField(as_device_tensor(other, self._t.device) + self.tensor)

    def __eq__(self, other):        # pragma: no cover - informational
        return NotImplemented

    __hash__ = object.__hash__

    def __repr__(self):
        return 'DeviceField(shape=%s, device=%s, pending=%d)' % (self.shape, self.device, self.pending)


def as_device_tensor(x, device=None):
    """The device tensor behind a field value (DeviceField, torch tensor or ndarray),
    queued exchange landed."""
    import torch
    if isinstance(x, DeviceField):
        return x.tensor
    t = torch.as_tensor(x, dtype=torch.float64)
    return t.to(device) if device is not None else t


def make_update_field_with_exchange(avogadro: float = N_A_LEGACY):
    """``update_field_with_exchange`` with N_A = ``avogadro`` (the reference reads
    scipy.constants.N_A, lattice_utils.py:15: 6.022140857e23 under the scipy its
    fixtures were made with)."""

    # every agent of a colony passes the same dimensions store values: their bin volume,
    # bin counts and the field shape they imply are derived once per set of values
    # (the entry holds the value objects, so identity stands for equality)
    last = [None]

    def derived(dims):
        n_bins, bounds, depth = dims['n_bins'], dims['bounds'], dims['depth']
        c = last[0]
        if c is None or c[0] is not n_bins or c[1] is not bounds or c[2] is not depth:
            nx, ny = int(n_bins[0]), int(n_bins[1])
            c = last[0] = (n_bins, bounds, depth, _bin_volume(n_bins, bounds, depth) * avogadro, nx, ny, (nx, ny))
        return c

    def update_field_with_exchange(current_value, new_value, states):
        location = states['global']['location']
        dims = states['dimensions']
        if type(current_value) is DeviceField:
            _, _, _, bva, nx, ny, shape = derived(dims)
            # get_bin_site (lattice_utils.py:18-40), as _bin_site: floor(loc * n / bound) % n
            i = int(math.floor(location[0] * nx / dims['bounds'][0])) % nx
            j = int(math.floor(location[1] * ny / dims['bounds'][1])) % ny
            if current_value._t.shape != shape:
                raise ValueError('field shape %s does not match n_bins %s' % (current_value.shape, [nx, ny]))
            current_value.queue_exchange(i * ny + j, int(new_value), bva)
            return current_value
        n_bins = dims['n_bins']
        bounds = dims['bounds']
        depth = dims['depth']
        i, j = _bin_site(location, n_bins, bounds)
        bva = _bin_volume(n_bins, bounds, depth) * avogadro
        if isinstance(current_value, DeviceField) or getattr(current_value, 'is_cuda', False):
            field = current_value if isinstance(current_value, DeviceField) else DeviceField(current_value)
            if field.shape != (int(n_bins[0]), int(n_bins[1])):
                raise ValueError('field shape %s does not match n_bins %s' % (field.shape, list(n_bins)))
            field.queue_exchange(i * int(n_bins[1]) + j, int(new_value), bva)
            return field
        # a host field: the reference's arithmetic (registry.py:173-183)
        delta = np.zeros((n_bins[0], n_bins[1]), dtype=np.float64)
        delta[i, j] += new_value / bva * 1000.0
        return current_value + delta

    def site(states):
        """(linear bin, bin_volume * N_A, field shape) of the agent whose port
        states are ``states`` -- what one call above derives for a DeviceField, for
        a caller that queues several molecules of one agent at once."""
        location = states['global']['location']
        dims = states['dimensions']
        _, _, _, bva, nx, ny, shape = derived(dims)
        i = int(math.floor(location[0] * nx / dims['bounds'][0])) % nx
        j = int(math.floor(location[1] * ny / dims['bounds'][1])) % ny
        return i * ny + j, bva, shape

    update_field_with_exchange.avogadro = avogadro
    update_field_with_exchange.site = site
    return update_field_with_exchange


#: the drop-in for registry.update_field_with_exchange (N_A of the reference fixtures)
update_field_with_exchange = make_update_field_with_exchange()


def flush_all(tree):
    """Land the queued exchange of every DeviceField in a nested dict (e.g. a
    store's state before a host snapshot); returns the tree."""
    if isinstance(tree, DeviceField):
        tree.flush()
    elif isinstance(tree, dict):
        for v in tree.values():
            flush_all(v)
    return tree
