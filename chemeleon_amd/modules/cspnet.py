"""CSPNet score network — same constructor, submodule names, state_dict keys
and forward contract as the reference `chemeleon/modules/cspnet.py:184-405`,
with the forward pass executed by the HIP library (`chm_decoder_forward`).

The nn.Modules below only hold parameters so that `load_state_dict` of a
reference checkpoint (keys under `decoder.`) works unchanged; all arithmetic
runs in hand-written gfx950 kernels. There is no CPU fallback: calling
forward with CPU tensors raises.
"""

import ctypes
import math
import threading
from collections import namedtuple
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from chemeleon_amd import _lib

_MATH_CODES = {"bf16x3": _lib.MATH_BF16X3, "f32": _lib.MATH_F32, "split16": _lib.MATH_SPLIT16}

DECODER_OUTPUTS = namedtuple("DECODER_OUTPUTS", ["atom_types_out", "lattice_out", "coords_out", "node_features"])


class SinusoidalTimeEmbeddings(nn.Module):
    """cspnet.py:21-35. Evaluated once per timestep table on the host; the
    sampler keeps the [T+1, dim] table on the device."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, time):
        half = self.dim // 2
        e = math.log(10000) / (half - 1)
        e = torch.exp(torch.arange(half, device=time.device) * -e)
        e = time[:, None] * e[None, :]
        return torch.cat((e.sin(), e.cos()), dim=-1)


class SinusoidsEmbedding(nn.Module):
    """cspnet.py:38-52 (parameter-free; computed in the `k_fourier` kernel)."""

    def __init__(self, n_frequencies=10, n_space=3):
        super().__init__()
        self.n_frequencies = n_frequencies
        self.n_space = n_space
        self.dim = n_frequencies * 2 * n_space


class FilmLayer(nn.Module):
    """Parameter container of cspnet.py:55-97 (FiLM over time + text)."""

    def __init__(self, hidden_dim=128, time_dim=256, text_dim=128, act_fn=None):
        super().__init__()
        self.hidden_dim, self.time_dim, self.text_dim = hidden_dim, time_dim, text_dim
        self.mlp_cond = nn.Sequential(nn.Linear(time_dim + text_dim, hidden_dim * 2), nn.SiLU())
        self.proj = nn.Linear(hidden_dim, hidden_dim)
        self.norm = nn.LayerNorm(hidden_dim)


class CSPLayer(nn.Module):
    """Parameter container of cspnet.py:100-181 (edge MLP, node MLP, LayerNorm)."""

    def __init__(self, hidden_dim=128, act_fn=None, dis_emb=None, ln=False, ip=True):
        super().__init__()
        self.dis_dim = dis_emb.dim if dis_emb is not None else 3
        self.ip = ip
        self.edge_mlp = nn.Sequential(nn.Linear(hidden_dim * 2 + 9 + self.dis_dim, hidden_dim), nn.SiLU(),
                                      nn.Linear(hidden_dim, hidden_dim), nn.SiLU())
        self.node_mlp = nn.Sequential(nn.Linear(hidden_dim * 2, hidden_dim), nn.SiLU(),
                                      nn.Linear(hidden_dim, hidden_dim), nn.SiLU())
        self.ln = ln
        if ln:
            self.layer_norm = nn.LayerNorm(hidden_dim)


class _HipModel:
    """Owns a chm_model (packed device weights)."""

    def __init__(self, net: "CSPNet"):
        L = _lib.load()
        params = [p.detach().float().contiguous() for p in net.ordered_parameters()]
        _lib.require_device(*params)
        dims = net.chm_dims()
        arr = (_lib.c_void_p * len(params))(*[p.data_ptr() for p in params])
        h = _lib.c_void_p()
        _lib.check(L.chm_model_create(dims, arr, len(params), _lib.stream_handle(params[0].device), h),
                   "chm_model_create")
        self.handle = h
        self.device = params[0].device

    def __del__(self):
        try:
            if self.handle:
                _lib.load().chm_model_destroy(self.handle)
        except Exception:
            pass


class HipBatch:
    """Owns a chm_batch: index tables of the fc edge layout + the decoder workspace.

    The workspace is a uint8 tensor from the PyTorch caching allocator, allocated on the
    stream that is current at creation (chm_batch_create_with_workspace), so its memory is
    budgeted with the rest of the process's device tensors. A batch is scratch for one stream:
    CSPNet.hip_batch keys its cache by stream."""

    def __init__(self, model: _HipModel, natoms, max_pairs: int, knn: bool = False, max_neighbors: int = 20,
                 knn_edges_per_atom: int = 128):
        L = _lib.load()
        nat = [int(n) for n in natoms]
        arr = (ctypes.c_int32 * len(nat))(*nat)
        opts = _lib.chm_batch_options(_lib.EDGES_KNN if knn else _lib.EDGES_FC, int(max_neighbors),
                                      int(knn_edges_per_atom), 0)
        need = int(L.chm_batch_workspace_bytes_ex(model.handle, arr, len(nat), max_pairs, ctypes.byref(opts)))
        if need == 0:
            _lib.check(-1, "chm_batch_workspace_bytes_ex")
        h = _lib.c_void_p()
        with torch.cuda.device(model.device):
            # 256-byte alignment: the caching allocator returns 512-byte aligned blocks
            self.workspace = torch.empty(need, dtype=torch.uint8, device=model.device)
            _lib.check(L.chm_batch_create_ex(model.handle, arr, len(nat), max_pairs, ctypes.byref(opts),
                                             _lib.ptr(self.workspace), need, _lib.stream_handle(model.device), h),
                       "chm_batch_create_ex")
        self.knn = bool(knn)
        self.handle = h
        self.model = model  # keep the weights alive
        self.natoms = tuple(nat)
        self.num_graphs = len(nat)
        self.num_nodes = int(L.chm_batch_num_nodes(h))
        self.num_edges = int(L.chm_batch_num_edges(h))
        self.device_bytes = int(L.chm_batch_device_bytes(h))
        self.max_pairs = max_pairs

    def __del__(self):
        try:
            if self.handle:
                _lib.load().chm_batch_destroy(self.handle)
        except Exception:
            pass


class CSPNet(nn.Module):
    def __init__(self, hidden_dim=128, time_dim=256, text_dim=128, num_layers=4, max_atoms=103, act_fn="silu",
                 dis_emb="sin", num_freqs=10, edge_style="fc", cutoff=6.0, max_neighbors=20, ln=False, ip=True,
                 smooth=True, pred_atom_types=True):
        super().__init__()
        self.hidden_dim, self.time_dim, self.text_dim = hidden_dim, time_dim, text_dim
        self.max_atoms, self.num_freqs = max_atoms, num_freqs
        self.ip, self.smooth, self.ln = ip, smooth, ln
        self.edge_style, self.cutoff, self.max_neighbors = edge_style, cutoff, max_neighbors
        self.pred_atom_types = pred_atom_types
        if smooth:
            self.node_embedding = nn.Linear(max_atoms, hidden_dim)
        else:
            self.node_embedding = nn.Embedding(max_atoms, hidden_dim)
        if time_dim > 0 or text_dim > 0:
            self.film_layer = FilmLayer(hidden_dim, time_dim, text_dim)
        if act_fn != "silu":
            raise ValueError("only act_fn='silu' exists in the reference")
        self.dis_emb = SinusoidsEmbedding(n_frequencies=num_freqs) if dis_emb == "sin" else None
        for i in range(num_layers):
            self.add_module(f"csp_layer_{i}", CSPLayer(hidden_dim, None, self.dis_emb, ln=ln, ip=ip))
        self.num_layers = num_layers
        self.coord_out = nn.Linear(hidden_dim, 3, bias=False)
        self.lattice_out = nn.Linear(hidden_dim, 9, bias=False)
        self.type_out = nn.Linear(hidden_dim, max_atoms)
        if ln:
            self.final_layer_norm = nn.LayerNorm(hidden_dim)
        self._hip: Optional[_HipModel] = None
        self._hip_sig = None
        self._batches: Dict[Tuple, HipBatch] = {}
        self._math: Optional[str] = None  # set_math choice, re-applied when the packed weights are rebuilt
        self._options: Dict[str, int] = {}  # set_option choices, likewise
        self._hip_lock = threading.RLock()

    # ------------------------------------------------------------------ HIP plumbing
    def chm_dims(self):
        return _lib.chm_dims(self.hidden_dim, self.time_dim, self.text_dim, self.num_layers, self.max_atoms,
                             self.num_freqs)

    def _check_supported(self):
        why = []
        if self.edge_style not in ("fc", "knn"):
            why.append(f"edge_style={self.edge_style!r}")
        if self.smooth:
            why.append("smooth=True")
        if not self.ln or not self.ip:
            why.append("ln=False / ip=False")
        if self.dis_emb is None:
            why.append("dis_emb='none'")
        if why:
            raise NotImplementedError("chemeleon_amd implements the shipped configuration only: " + ", ".join(why))

    def ordered_parameters(self):
        """Parameters in the order of the C ABI (= state_dict order)."""
        return [v for k, v in self.state_dict(keep_vars=True).items()]

    def hip_model(self) -> _HipModel:
        self._check_supported()
        with self._hip_lock:
            sig = tuple((p.data_ptr(), p._version, str(p.device)) for p in self.parameters())
            if self._hip is None or sig != self._hip_sig:
                self._hip = _HipModel(self)
                self._hip_sig = sig
                self._batches.clear()
                if self._math is not None:
                    _lib.check(_lib.load().chm_model_set_math(self._hip.handle, _MATH_CODES[self._math]),
                               "chm_model_set_math")
                for k, v in self._options.items():
                    _lib.check(_lib.load().chm_model_set_option(self._hip.handle, k.encode(), int(v)),
                               "chm_model_set_option")
            return self._hip

    def set_option(self, key: str, value: int):
        """Launch-schedule option of the C ABI (chm_model_set_option, e.g. 'edge_split'); results are
        bit-identical either way. Survives rebuilds of the packed weights."""
        with self._hip_lock:
            _lib.check(_lib.load().chm_model_set_option(self.hip_model().handle, key.encode(), int(value)),
                       "chm_model_set_option")
            self._options[key] = int(value)
            # (a batch carves the pre-split operand buffers only when created with node_ps, plans its
            # pair-grid job lists with the edge_lag of its creation and picks its row tiling (short last-round
            # tiles or the one-grid schedules' uniform ones) from the options of its creation: cached batches
            # are rebuilt)
            if key in ("node_ps", "edge_lag", "edge_layer_min", "edge_rows_short", "edge_rows"):
                self._batches.clear()

    def set_math(self, mode: str):
        """'split16' (default), 'bf16x3' or 'f32' for the decoder GEMMs (see include/chemeleon_hip.h).
        The choice survives rebuilds of the packed weights (load_state_dict, .to())."""
        code = _MATH_CODES[mode]
        with self._hip_lock:
            m = self.hip_model()
            _lib.check(_lib.load().chm_model_set_math(m.handle, code), "chm_model_set_math")
            self._math = mode
            self._batches.clear()

    def get_math(self) -> str:
        return {0: "bf16x3", 1: "f32", 2: "split16"}[_lib.load().chm_model_get_math(self.hip_model().handle)]

    def hip_batch(self, natoms, max_pairs: int = 1, stream=None, private: bool = False) -> HipBatch:
        """Workspace + edge tables for this crystal list, cached per (natoms, max_pairs, stream):
        concurrent samplers on different streams never share scratch. private=True returns a
        fresh, uncached batch (one per concurrent lane of a captured step)."""
        m = self.hip_model()
        nat = tuple(int(n) for n in natoms)
        knn = dict(knn=self.edge_style == "knn", max_neighbors=self.max_neighbors)
        if private:
            return HipBatch(m, nat, max_pairs, **knn)
        if stream is None:
            stream = torch.cuda.current_stream(m.device)
        key = (nat, max_pairs, int(stream.cuda_stream))
        with self._hip_lock:
            b = self._batches.get(key)
            if b is None:
                if len(self._batches) >= 4:
                    self._batches.pop(next(iter(self._batches)))
                with torch.cuda.stream(stream):
                    b = HipBatch(m, nat, max_pairs, **knn)
                self._batches[key] = b
            return b

    # ------------------------------------------------------------------ forward
    def _run(self, pairs, atom_types, frac_coords, lattices, num_atoms, t, text, need_nodes=True):
        film = self.time_dim > 0 or self.text_dim > 0
        if t is None and film:
            raise NotImplementedError("time embeddings are required (the sampling path always passes them)")
        natoms = num_atoms.tolist() if torch.is_tensor(num_atoms) else list(num_atoms)
        b = self.hip_batch(natoms, max_pairs=max(pairs, 1))
        dev = self.hip_model().device
        a = atom_types.long().contiguous()
        x = frac_coords.float().contiguous()
        lat = lattices.float().contiguous()
        te = t.float().contiguous() if film else None  # (no FilmLayer: time and text are not used)
        tx = text.float().contiguous() if text is not None and film else None
        _lib.require_device(a, x, lat, te, tx)
        B, N = b.num_graphs, b.num_nodes
        if a.shape[0] != N or x.shape != (N, 3) or lat.shape != (B, 3, 3) or (film and te.shape != (B, self.time_dim)):
            raise ValueError("decoder input shapes do not match num_atoms")
        if self.text_dim > 0 and (tx is None or tx.shape[-1] != self.text_dim):
            raise ValueError("text embeddings of width text_dim are required")
        types = torch.empty(pairs, N, self.max_atoms, device=dev)
        latt = torch.empty(pairs, B, 3, 3, device=dev)
        coords = torch.empty(pairs, N, 3, device=dev)
        nodes = torch.empty(pairs, N, self.hidden_dim, device=dev) if need_nodes else None
        L = _lib.load()
        _lib.check(L.chm_decoder_forward(b.handle, pairs, _lib.ptr(a), _lib.ptr(x), _lib.ptr(lat), _lib.ptr(te),
                                         self.time_dim, _lib.ptr(tx), _lib.ptr(types), _lib.ptr(latt),
                                         _lib.ptr(coords), _lib.ptr(nodes), _lib.stream_handle(dev)),
                   "chm_decoder_forward")
        return types, latt, coords, nodes

    def forward(self, atom_types, frac_coords, lattices, num_atoms, node2graph, t=None, text_embeds=None):
        """cspnet.py:345-405. node2graph must be `arange(B).repeat_interleave(num_atoms)`
        (what Batch.from_data_list builds); the graph layout is taken from num_atoms."""
        types, latt, coords, nodes = self._run(1, atom_types, frac_coords, lattices, num_atoms, t, text_embeds)
        return DECODER_OUTPUTS(atom_types_out=types[0] if self.pred_atom_types else None, lattice_out=latt[0],
                               coords_out=coords[0], node_features=nodes[0])

    def forward_cfg(self, atom_types, frac_coords, lattices, num_atoms, t, text_cond, text_null, need_nodes=False):
        """The two decoder calls of Chemeleon.model_predictions (chemeleon.py:258-285)
        as ONE batched call: cond / null share atoms, coordinates, lattices and
        the Fourier edge projection. Returns (types, lattice, coords, nodes),
        each with a leading [2] axis (0 = cond, 1 = null)."""
        text = torch.stack([text_cond.float(), text_null.float()], 0).contiguous()
        return self._run(2, atom_types, frac_coords, lattices, num_atoms, t, text, need_nodes)
