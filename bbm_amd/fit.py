"""Fitting on the GPU: linearizers, sampled losses and the compass search (BASELINE config 5).

Host-side mirror of the reference's fitting layer (include/bbm/sampledlossfunction.h,
include/loss/*.h, include/linearizer/*.h, include/optimizer/compass.h):

* `spherical_linearizer` / `merl_linearizer` describe the (in, out) sample grid
  (bbm_hip_linearizer, include/bbm_hip.h);
* `SampledLoss(fitted, reference, loss, linearizer)` is sampledlossfunction: the mean of a
  per-sample loss (nganL2 ... bieronLog) between the fitted model and a reference over the grid.
  The reference is a table of RGB values on the grid (a measured material is a table); it can be
  filled from a model on the GPU (`reference_table`).  `probe_losses(P)` evaluates many parameter
  vectors in ONE kernel launch (bbm_hip_loss) -- the 2P probes of a compass step;
* `Compass` is compass (compass.h:40-183) with the probes batched: the host reproduces the
  reference's sequence of float parameter updates exactly (probe, restore by subtraction, box
  test), the GPU scores all probes of the step at once, and the host applies the reference's
  sequential "strictly better" rule to the scores.

Multi-GPU (one process per GPU, torch.distributed): the sample grid is split into contiguous
shards; every rank scores all probes on its shard and the per-probe sums are all-reduced (RCCL
over xGMI, 2P doubles per step).  Every rank then takes the identical compass decision.
"""
import ctypes
import math

import numpy as np

from . import _lib
from .backbone import AggregateModel, _on_stream, _stream_ptr, _torch, tree_desc

LIN_SPHERICAL, LIN_MERL = 0, 1
NGAN_L2, LOW_L2, BIERON_L2, STANDARD_LOG, LOW_LOG, BIERON_LOG = range(6)
LOSS_NAMES = {"nganL2": NGAN_L2, "lowL2": LOW_L2, "bieronL2": BIERON_L2, "standardLog": STANDARD_LOG,
              "lowLog": LOW_LOG, "bieronLog": BIERON_LOG}
ALL = 0x0F          # bsdf_attr::All (include/bbm/bsdf_attr_flag.h:27)

_F32 = np.float32
# constants<float>::Pi(scale) = T(scale * std::numbers::pi) (include/core/constants.h:16-24)
PI = float(_F32(math.pi))
HEMISPHERE = (float(_F32(2.0 * math.pi)), float(_F32(0.5 * math.pi)))
EPSILON = float(np.finfo(np.float32).eps)


class Linearizer(ctypes.Structure):
    """bbm_hip_linearizer (include/bbm_hip.h)."""
    _fields_ = [("kind", ctypes.c_int32), ("samples_in", ctypes.c_uint64 * 2), ("samples_out", ctypes.c_uint64 * 2),
                ("start_in", ctypes.c_float * 2), ("end_in", ctypes.c_float * 2),
                ("start_out", ctypes.c_float * 2), ("end_out", ctypes.c_float * 2)]

    def size(self):
        n = ctypes.c_uint64()
        _lib.check(_lib.load().bbm_hip_linearizer_size(ctypes.byref(self), ctypes.byref(n)))
        return int(n.value)

    def directions(self, begin=0, n=None, stream=None):
        """(in, out) direction pairs begin .. begin+n-1 -> two (3, n) float32 CUDA tensors."""
        torch = _torch()
        if n is None:
            n = self.size() - begin
        dev = torch.device("cuda", torch.cuda.current_device())
        din = torch.empty((3, n), dtype=torch.float32, device=dev)
        dout = torch.empty((3, n), dtype=torch.float32, device=dev)
        _lib.check(_lib.load().bbm_hip_linearize(ctypes.byref(self), begin, n, din[0].data_ptr(), din[1].data_ptr(),
                                                  din[2].data_ptr(), dout[0].data_ptr(), dout[1].data_ptr(),
                                                  dout[2].data_ptr(), _stream_ptr(stream)))
        return din, dout


def spherical_linearizer(samples_in, samples_out, start_in=(0.0, 0.0), end_in=HEMISPHERE, start_out=(0.0, 0.0),
                         end_out=HEMISPHERE):
    """spherical_linearizer(samplesIn, samplesOut, startIn, endIn, startOut, endOut), all (phi, theta)
    (include/linearizer/spherical_linearizer.h:38-45)."""
    lin = Linearizer()
    lin.kind = LIN_SPHERICAL
    for k in range(2):
        lin.samples_in[k], lin.samples_out[k] = int(samples_in[k]), int(samples_out[k])
        lin.start_in[k], lin.end_in[k] = start_in[k], end_in[k]
        lin.start_out[k], lin.end_out[k] = start_out[k], end_out[k]
    return lin


def merl_linearizer(h=(1, 90), d=(180, 90)):
    """merl_linearizer(samplesH, samplesD) (include/linearizer/merl_linearizer.h:28)."""
    lin = Linearizer()
    lin.kind = LIN_MERL
    for k in range(2):
        lin.samples_in[k], lin.samples_out[k] = int(h[k]), int(d[k])
    return lin


def shard_range(total, rank, world):
    """Contiguous shard [begin, end) of `total` samples for `rank` of `world` (balanced)."""
    q, r = divmod(total, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def reference_table(model, lin, begin=0, n=None, stream=None):
    """Reference values on the linearizer's samples begin .. begin+n-1: model.eval on the GPU
    (Spectrum per sample, component All) -> (3, n) float32 CUDA tensor."""
    din, dout = lin.directions(begin, n, stream)
    return model.eval(din, dout, stream=stream)


class SampledLoss:
    """sampledlossfunction<fitted, reference, loss, linearizer> (include/bbm/sampledlossfunction.h:34-97).

    fitted: any model -- a BsdfModel (one fused kernel: bbm_hip_loss / bbm_hip_loss_pairs, all probes in one launch)
    or an AggregateModel of any composition (composed aggregates and runtime aggregates: bbm_hip_loss_tree, the
    probes evaluated through the children's kernels) -- whose parameter layout the probes use; reference: a model
    (evaluated once into a table on this rank's shard) or a (3, n_shard) CUDA tensor of reference values.
    f64: the doubleRGB configuration (bbm_hip_loss_tree_f64: directions, reference values, parameters and
    per-sample losses in double).  dist: torch.distributed module (or None); the shard is this rank's part of the
    grid."""

    def __init__(self, fitted, reference, loss, lin=None, component=3, unit=0, dist=None, stream=None, materialize=True,
                 f64=False, pairs=None):
        torch = _torch()
        self.f64 = bool(f64)
        # the fused multi-probe kernel serves single floatRGB models; everything else the materialised tree path
        self.tree = self.f64 or isinstance(fitted, AggregateModel)
        if self.tree:
            materialize = True
            if self.f64 and not fitted.has_f64():
                raise _lib.BackboneError(_lib.ERR_UNSUPPORTED, f"{fitted.name}: no doubleRGB kernels")
        self.fitted = fitted
        self.loss_kind = LOSS_NAMES[loss] if isinstance(loss, str) else int(loss)
        self.lin = lin
        self.component, self.unit = int(component), int(unit)
        self.dist = dist
        self.stream = stream
        if pairs is not None:
            # a table of direction pairs (this rank's own samples: the reference's sampledlossfunction over any
            # linearizer, e.g. the measured directions of a material) instead of a grid
            self.pairs = tuple(pairs)
            self.n = self.total = int(self.pairs[0].shape[1])
            self.begin = 0
            if dist is not None and dist.get_world_size() > 1:
                # every rank holds its own pairs: the grid is their concatenation in rank order (total = the sum of
                # the counts, this rank's samples start after the lower ranks'), so the losses are means over all
                counts = _torch().zeros(dist.get_world_size(), dtype=_torch().int64, device=self.pairs[0].device)
                counts[dist.get_rank()] = self.n
                dist.all_reduce(counts)
                counts = counts.cpu().tolist()
                self.total = int(sum(counts))
                self.begin = int(sum(counts[:dist.get_rank()]))
        else:
            self.total = lin.size()
            rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
            self.begin, end = shard_range(self.total, rank, world)
            self.n = end - self.begin
            # materialize: the shard's direction pairs are computed once (bbm_hip_linearize, 24 B/sample resident)
            # and every compass step streams them (bbm_hip_loss_pairs) instead of recomputing the linearizer
            self.pairs = lin.directions(self.begin, self.n, stream) if materialize else None
        if self.f64:
            self.pairs = tuple(d.double() for d in self.pairs)
        if hasattr(reference, "eval"):
            if self.pairs is not None:
                self.ref = reference.eval(self.pairs[0], self.pairs[1], stream=stream)
            else:
                self.ref = reference_table(reference, lin, self.begin, self.n, stream)
        else:
            self.ref = reference
        if self.f64:
            self.ref = self.ref.double()
        if self.ref.shape != (3, self.n):
            raise ValueError(f"reference table: expected shape (3, {self.n}), got {tuple(self.ref.shape)}")
        self.dev = self.ref.device
        self._ws = None
        self._ws_probes = 0
        self.launches = 0

    def update(self):
        """sampledlossfunction::update() (sampledlossfunction.h:52): nothing to refresh."""

    def _sample_loss(self, idx, params=None):
        if not 0 <= idx < self.total:
            return 0.0
        return Batch._one(self, idx, params)

    def samples(self):
        return self.total

    def materialized(self):
        """This rank's shard as (pairs, reference table, n).  A loss that streams its pairs from the linearizer
        (materialize=False) computes them into a temporary the caller holds (24 B per sample while it lives): the loss
        itself stays on the streaming kernel and keeps no copy."""
        pairs = self.pairs if self.pairs is not None else self.lin.directions(self.begin, self.n, self.stream)
        return pairs, self.ref, self.n

    def _workspace(self, nprobes, n=None):
        torch = _torch()
        lib = _lib.load()
        nbytes = (lib.bbm_hip_loss_tree_workspace_size(nprobes, self.n if n is None else n) if self.tree
                  else lib.bbm_hip_loss_workspace_size(nprobes))
        if self._ws is None or self._ws.numel() * 8 < nbytes:
            self._ws = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=self.dev)
            self._ws_probes = nprobes
        return self._ws

    def probe_sums(self, probes, pairs=None, ref=None, n=None):
        """Per-probe loss sums over the WHOLE grid: this rank's shard (local_sums), then the
        cross-rank all-reduce -- RCCL over xGMI, 2P doubles per compass step."""
        sums = self.local_sums(probes) if pairs is None else self.local_sums(probes, pairs, ref, n)
        if self.dist is not None and self.dist.get_world_size() > 1:
            torch = _torch()
            stream = getattr(self, "stream", None)
            if stream is not None and sums.is_cuda:
                # the collective runs on the current stream: order it after the loss launch on self.stream
                torch.cuda.current_stream().wait_stream(stream)
            self.dist.all_reduce(sums)
        return sums

    def _tree_sums(self, probes, pairs=None, ref=None, n=None):
        """bbm_hip_loss_tree(_f64): any model, probes on the host; over this rank's shard, or over the given pairs /
        reference table of n samples (a batch's gathered samples)."""
        torch = _torch()
        if pairs is None:
            pairs, ref, n = self.pairs, self.ref, self.n
        npar = self.fitted.parameter_values().size
        p = np.ascontiguousarray(np.asarray(probes, dtype=np.float64 if self.f64 else np.float32).reshape(-1, npar))
        nprobes = p.shape[0]
        sums = torch.empty(nprobes, dtype=torch.float64, device=self.dev)
        if n == 0:
            return sums.zero_()
        ws = self._workspace(nprobes, n)
        _on_stream(self.stream, sums, ws)
        tree, ntree, _keep = tree_desc(self.fitted, self.f64)
        lib = _lib.load()
        fn = lib.bbm_hip_loss_tree_f64 if self.f64 else lib.bbm_hip_loss_tree
        din, dout = pairs
        _lib.check(fn(tree, ntree, p.ctypes.data, npar, nprobes, n, din[0].data_ptr(), din[1].data_ptr(),
                      din[2].data_ptr(), dout[0].data_ptr(), dout[1].data_ptr(), dout[2].data_ptr(),
                      ref[0].data_ptr(), ref[1].data_ptr(), ref[2].data_ptr(), self.loss_kind,
                      self.component, self.unit, sums.data_ptr(), ws.data_ptr(), ws.numel() * 8,
                      _stream_ptr(self.stream)))
        self.launches += 1
        return sums

    def local_sums(self, probes, pairs=None, ref=None, n=None):
        """Per-probe loss sums over this rank's shard (or over the given pairs / reference table of n samples): one
        bbm_hip_loss launch -> float64 tensor (nprobes,)."""
        if self.tree:
            return self._tree_sums(probes, pairs, ref, n)
        torch = _torch()
        if pairs is None:
            pairs, ref, n = self.pairs, self.ref, self.n
        p = np.ascontiguousarray(np.asarray(probes, dtype=np.float32).reshape(-1, self.fitted._params.size))
        nprobes, npar = p.shape
        dp = torch.from_numpy(p).to(self.dev, non_blocking=False)
        sums = torch.empty(nprobes, dtype=torch.float64, device=self.dev)
        if n == 0:
            return sums.zero_()
        ws = self._workspace(nprobes)
        _on_stream(self.stream, dp, sums, ws)
        lib = _lib.load()
        if pairs is not None:
            din, dout = pairs
            _lib.check(lib.bbm_hip_loss_pairs(self.fitted.model_id, dp.data_ptr(), npar, nprobes, n,
                                              din[0].data_ptr(), din[1].data_ptr(), din[2].data_ptr(),
                                              dout[0].data_ptr(), dout[1].data_ptr(), dout[2].data_ptr(),
                                              ref[0].data_ptr(), ref[1].data_ptr(), ref[2].data_ptr(),
                                              self.loss_kind, self.component, self.unit, sums.data_ptr(), ws.data_ptr(),
                                              ws.numel() * 8, _stream_ptr(self.stream)))
        else:
            _lib.check(lib.bbm_hip_loss(self.fitted.model_id, dp.data_ptr(), npar, nprobes, ctypes.byref(self.lin),
                                        self.begin, self.n, self.ref[0].data_ptr(), self.ref[1].data_ptr(),
                                        self.ref[2].data_ptr(), self.loss_kind, self.component, self.unit,
                                        sums.data_ptr(), ws.data_ptr(), ws.numel() * 8, _stream_ptr(self.stream)))
        self.launches += 1
        return sums

    def probe_losses(self, probes):
        """Mean loss per probe (err / numsamples, sampledlossfunction.h:80-87) as Value: float32 values (float64 in
        doubleRGB)."""
        s = self.probe_sums(probes).cpu().numpy()
        return s / float(self.total) if getattr(self, "f64", False) else (s / float(self.total)).astype(np.float32)

    def __call__(self, arg=None, params=None):
        """Loss of one parameter vector `arg` (the fitted model's current parameters by default); with an integer
        `arg`, the loss of that sample alone (sampledlossfunction::operator()(idx), sampledlossfunction.h:62-73; 0
        past the last sample) at `params`."""
        if isinstance(arg, (int, np.integer)):
            return self._sample_loss(int(arg), params)
        params = arg if params is None else params
        p = self.fitted.parameter_values() if params is None else params
        f64 = getattr(self, "f64", False)
        return float(self.probe_losses(np.asarray(p, np.float64 if f64 else np.float32)[None])[0])


class BatchRng:
    """bbm::rng<Size_t> (backbone/native/include/backbone/random.h:40-66): std::mt19937_64 and libstdc++'s
    uniform_int_distribution over [lower, upper] (both ends included), restated in the library (bbm_hip_rng_*) so a
    batch draws the reference's indices for the same seed."""

    def __init__(self, seed=_lib.RNG_DEFAULT_SEED, lower=0, upper=2 ** 64 - 1):
        self.state = _lib.Rng()
        _lib.check(_lib.load().bbm_hip_rng_init(ctypes.byref(self.state), int(seed), int(lower), int(upper)))

    def draw(self, n):
        """The next n numbers -> (n,) uint64."""
        out = np.zeros(int(n), np.uint64)
        _lib.check(_lib.load().bbm_hip_rng_draw(ctypes.byref(self.state), out.ctypes.data, out.size))
        return out


class Batch:
    """bbm::batch<SAMPLEDLOSSFUNC> (include/bbm/batch.h:27-92): the loss over `batchsize` samples of a SampledLoss,
    drawn at random (with repetition) and redrawn by every update() -- compass calls update() once per step
    (compass.h:103), so each step scores its 2P probes on a fresh batch.

    Indices: bbm::rng<Size_t>(seed, 0, samples()) (batch.h:40), i.e. in [0, samples()] -- the last value is past the
    final sample and that lane's loss is 0 (sampledlossfunction.h:65-66).  The batch's samples are gathered from the
    materialised pairs and reference table (bbm_hip_gather_samples, one device pass per update) and all probes are
    scored in one launch of the inner loss's kernel.  Sharded losses (dist): each rank gathers the indices inside its
    own shard; the per-probe sums are all-reduced as for the whole grid.

    loss_value() / probe_losses(): sum over the batch / batchsize.  The reference's whole-batch operator()
    (batch.h:75-82) reads an uninitialised loop index (`for(size_t i; ...)`, undefined behaviour); this is the
    mean it was written to compute.  __call__(idx) is batch::operator()(idx) (batch.h:64-70)."""

    def __init__(self, batchsize, sampledloss, seed=_lib.RNG_DEFAULT_SEED):
        self.loss = sampledloss
        self.batchsize = int(batchsize)
        self.rng = BatchRng(seed, 0, sampledloss.samples())
        self.f64 = getattr(sampledloss, "f64", False)
        self.fitted = sampledloss.fitted
        self.index = np.zeros(self.batchsize, np.uint64)
        self._gathered = None
        self.update()

    def update(self):
        """batch.h:48-54: the wrapped loss's update(), then batchsize fresh indices."""
        self.loss.update()
        self.index = self.rng.draw(self.batchsize)
        self._gathered = None

    def samples(self):
        return self.batchsize

    def _gather(self, index):
        """This rank's samples among the global indices `index`, gathered densely -> (pairs, ref, n)."""
        torch = _torch()
        if getattr(self, "_shard", None) is None:
            # the shard's pairs for this batch's gathers (a temporary for a streaming loss, held by the batch only)
            self._shard = self.loss.materialized()
        pairs, ref, n = self._shard
        begin = self.loss.begin
        idx = np.asarray(index, np.uint64)
        mine = idx[(idx >= begin) & (idx < begin + n)] - np.uint64(begin)
        dt = torch.float64 if self.f64 else torch.float32
        dst = torch.empty((9, max(mine.size, 1)), dtype=dt, device=ref.device)
        src = [pairs[0][k] for k in range(3)] + [pairs[1][k] for k in range(3)] + [ref[k] for k in range(3)]
        src = [t.contiguous() for t in src]
        sp = (ctypes.c_void_p * 9)(*[t.data_ptr() for t in src])
        dp = (ctypes.c_void_p * 9)(*[dst[k].data_ptr() for k in range(9)])
        mine = np.ascontiguousarray(mine)
        lib = _lib.load()
        fn = lib.bbm_hip_gather_samples_f64 if self.f64 else lib.bbm_hip_gather_samples
        _on_stream(self.loss.stream, dst)
        got = _lib.check(fn(mine.ctypes.data, mine.size, n, ctypes.cast(sp, ctypes.c_void_p),
                            ctypes.cast(dp, ctypes.c_void_p), 9, _stream_ptr(self.loss.stream)))
        g = dst[:, :got]
        return (g[0:3], g[3:6]), g[6:9], int(got)

    def probe_sums(self, probes):
        """Per-probe loss sums over the current batch (all ranks), one launch -> float64 tensor (nprobes,)."""
        if self._gathered is None:
            self._gathered = self._gather(self.index)
        pairs, ref, n = self._gathered
        return self.loss.probe_sums(probes, pairs, ref, n)

    def probe_losses(self, probes):
        """Mean loss over the batch per probe, as Value (float32; float64 in doubleRGB)."""
        s = self.probe_sums(probes).cpu().numpy()
        return s / float(self.batchsize) if self.f64 else (s / float(self.batchsize)).astype(np.float32)

    def loss_value(self, params=None):
        p = self.fitted.parameter_values() if params is None else params
        return float(self.probe_losses(np.asarray(p, np.float64 if self.f64 else np.float32)[None])[0])

    def __call__(self, arg=None, params=None):
        """batch::operator()(idx) (batch.h:64-70) for an integer `arg`: the wrapped loss at the idx-th drawn index (0
        for idx >= batchsize and for the masked index samples()); otherwise the batch mean at parameters `arg`."""
        if not isinstance(arg, (int, np.integer)):
            return self.loss_value(arg if params is None else params)
        if not 0 <= int(arg) < self.batchsize:
            return 0.0
        i = int(self.index[int(arg)])
        return 0.0 if i >= self.loss.samples() else Batch._one(self.loss, i, params)

    @staticmethod
    def _one(loss, i, params):
        """The loss of global sample i alone at params, through a one-sample gather (sums over ranks: only the
        owner's is nonzero)."""
        p = loss.fitted.parameter_values() if params is None else params
        g = Batch.__new__(Batch)
        g.loss, g.f64 = loss, getattr(loss, "f64", False)
        pairs, ref, n = g._gather(np.asarray([i], np.uint64))
        dt = np.float64 if g.f64 else np.float32
        s = loss.probe_sums(np.asarray(p, dt)[None], pairs, ref, n).cpu().numpy()[0]
        return float(dt(s))


def _update(loss):
    """loss.update() where the loss has one (concepts::sampledlossfunction's update(), sampledlossfunction.h:52,
    batch.h:48-54); a loss object without it -- only probe_losses(probes) and __call__(params) -- needs none."""
    fn = getattr(loss, "update", None)
    if fn is not None:
        fn()


class Compass:
    """compass<LOSSFUNC, PARAM> (include/optimizer/compass.h:40-183), probes batched on the GPU.

    The loss protocol: probe_losses(probes) -> one loss per row of probes (a compass step's 2P probes in one call),
    __call__(params) -> the loss at one full parameter vector, and optionally update() (called before each step and
    by reset(), as compass.h:102-103 / :145-150 call the loss's).

    Optimises model.parameter_values(flag) (default bsdf_attr::All: Dependent attributes are held
    fixed) inside [lower, upper] (default: the model's parameter bounds); the model's parameters
    are updated in place, like the reference's parameter references."""

    def __init__(self, lossfunc, model=None, lower=None, upper=None, tolerance=None, step_size=1.0,
                 contraction=0.5, expansion=1.0, flag=ALL):
        self.loss = lossfunc
        self.model = model if model is not None else lossfunc.fitted
        # Value of the configuration: float32 (floatRGB) or float64 (the loss's doubleRGB), for every parameter,
        # step and loss the compass holds (compass.h:40-60 is templated on the parameter type)
        V = self.V = np.float64 if getattr(lossfunc, "f64", False) else _F32
        self.idx = self.model.parameter_indices(flag)
        full_lo = self.model.parameter_lower_bound()
        full_hi = self.model.parameter_upper_bound()
        self.lower = (np.asarray(lower, V) if lower is not None else full_lo[self.idx]).astype(V)
        self.upper = (np.asarray(upper, V) if upper is not None else full_hi[self.idx]).astype(V)
        # the full parameter vector the probes are built from (the model keeps float storage; in doubleRGB the
        # compass's double vector is the authoritative one, `parameters`)
        self.full = np.asarray(self.model.parameter_values(), V).copy()
        self.directions = []
        for i in range(1, len(self.idx) + 1):       # for(Scalar i=1; i <= size(param); ++i) (compass.h:67-71)
            self.directions += [float(i), -float(i)]
        eps = np.finfo(V).eps if tolerance is None else tolerance     # Constants::Epsilon() of the Value
        self.initial_step = V(step_size)
        self.tolerance = V(eps)
        self.contraction, self.expansion = V(contraction), V(expansion)
        self.reset()

    @property
    def parameters(self):
        """The current full parameter vector in the configuration's Value type."""
        return self.full.copy()

    def reset(self):
        """compass.h:145-150: step size back to the initial one, the loss's update(), loss of the current
        parameters."""
        self.step_size = self.initial_step
        _update(self.loss)
        self.loss_value = self.V(self.loss(self.full))

    def is_converged(self):
        return bool(self.step_size < self.tolerance)

    def _params(self):
        return self.full[self.idx].astype(self.V)

    def step(self):
        """One compass step (compass.h:82-140).  Returns the loss after the update."""
        V = self.V
        if self.is_converged():
            return V(0)
        _update(self.loss)                      # compass.h:102-103, before the probes
        param = self._params()
        s = self.step_size
        probes, in_box = [], []
        full = self.full.copy()
        for card in self.directions:
            k = int(abs(card)) - 1
            # probe(cardinal): value = param[k] + (cardinal < 0 ? -step : step), Value arithmetic
            param[k] = V(param[k] + (-s if card < 0 else s))
            inb = bool(np.all((param >= self.lower) & (param <= self.upper)))
            full[self.idx] = param
            probes.append(full.copy())
            in_box.append(inb)
            # probe(-cardinal): the reference restores by the opposite update (not by assignment)
            param[k] = V(param[k] + (s if card < 0 else -s))
        probes = np.stack(probes)
        in_box = np.asarray(in_box)
        errs = np.zeros(len(probes), V)
        if in_box.any():
            errs[in_box] = self.loss.probe_losses(probes[in_box])
        # sequential selection of the strictly best in-box probe (compass.h:118-121)
        best, loss = 0.0, self.loss_value
        for card, inb, err in zip(self.directions, in_box, errs):
            if inb and err < loss:
                best, loss = card, err
        optimize = bool(loss < self.loss_value)
        if optimize and best != 0:
            k = int(abs(best)) - 1
            param[k] = V(param[k] + (-s if best < 0 else s))
        # the parameters keep any round-off of the probe/restore sequence, as the reference's do
        self.full[self.idx] = param
        self.model.set_parameter_values(self.full)
        self.step_size = V(self.expansion * s) if optimize else V(self.contraction * s)
        if optimize:
            self.loss_value = V(loss)
        return self.loss_value
