"""Trajectory containers and structure output (reference
`chemeleon/modules/schema.py:14-88`).

`get_atoms` returns `ase.Atoms` when ase is importable, otherwise a minimal
`Atoms` with the same fields the reference callers use (numbers, cell, pbc,
scaled positions, chemical symbols / formula). In both cases the atoms of
each structure are sorted by chemical symbol (stable), as
`ase.build.tools.sort` does in the reference (schema.py:81).
"""

from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Union

import numpy as np
import torch

CHEMICAL_SYMBOLS = (
    "X H He Li Be B C N O F Ne Na Mg Al Si P S Cl Ar K Ca Sc Ti V Cr Mn Fe Co Ni Cu Zn Ga Ge As Se "
    "Br Kr Rb Sr Y Zr Nb Mo Tc Ru Rh Pd Ag Cd In Sn Sb Te I Xe Cs Ba La Ce Pr Nd Pm Sm Eu Gd Tb Dy Ho "
    "Er Tm Yb Lu Hf Ta W Re Os Ir Pt Au Hg Tl Pb Bi Po At Rn Fr Ra Ac Th Pa U Np Pu Am Cm Bk Cf Es Fm "
    "Md No Lr"
).split()

try:  # pragma: no cover - ase is not installed in this image
    from ase import Atoms as _AseAtoms
    from ase.build.tools import sort as _ase_sort
except Exception:  # noqa: BLE001
    _AseAtoms = None
    _ase_sort = None


class Atoms:
    """Minimal stand-in for ase.Atoms (used only when ase is unavailable)."""

    def __init__(self, numbers, cell, pbc=True, scaled_positions=None):
        self.numbers = np.asarray(numbers, dtype=np.int64)
        self.cell = np.asarray(cell, dtype=np.float64).reshape(3, 3)
        self.pbc = pbc
        self._scaled = (np.zeros((len(self.numbers), 3)) if scaled_positions is None
                        else np.asarray(scaled_positions, dtype=np.float64))

    def __len__(self):
        return len(self.numbers)

    def set_scaled_positions(self, p):
        self._scaled = np.asarray(p, dtype=np.float64)

    def get_scaled_positions(self, wrap=True):
        return self._scaled.copy()

    def get_positions(self):
        return self._scaled @ self.cell

    def get_atomic_numbers(self):
        return self.numbers.copy()

    def get_chemical_symbols(self):
        return [CHEMICAL_SYMBOLS[int(z)] for z in self.numbers]

    def get_chemical_formula(self):
        syms = self.get_chemical_symbols()
        return "".join(f"{s}{syms.count(s) if syms.count(s) > 1 else ''}" for s in sorted(set(syms)))

    def __getitem__(self, idx):
        return Atoms(self.numbers[idx], self.cell, self.pbc, self._scaled[idx])

    def __repr__(self):
        return f"Atoms(symbols='{self.get_chemical_formula()}', pbc={self.pbc})"


def sort_atoms(atoms):
    """ase.build.tools.sort: stable sort by chemical symbol."""
    if _ase_sort is not None and not isinstance(atoms, Atoms):
        return _ase_sort(atoms)
    tags = atoms.get_chemical_symbols()
    order = [i for _, i in sorted((tag, i) for i, tag in enumerate(tags))]
    return atoms[order]


def make_atoms(numbers, cell, scaled):
    if _AseAtoms is not None:
        at = _AseAtoms(numbers=numbers, cell=cell, pbc=True)
        at.set_scaled_positions(scaled)
        return at
    return Atoms(numbers, cell, True, scaled)


@dataclass
class TrajectoryStep:
    """schema.py:14-24"""
    num_atoms: torch.Tensor
    atom_types: torch.Tensor
    frac_coords: torch.Tensor
    lattices: torch.Tensor
    batch_idx: torch.Tensor
    atom_types_probs: Optional[torch.Tensor] = None


class TrajectoryContainer:
    """schema.py:26-88: time step -> TrajectoryStep."""

    def __init__(self, total_steps: int):
        self.total_steps = total_steps
        self.trajectory_continaer: Dict[int, Optional[TrajectoryStep]] = OrderedDict(
            (t, None) for t in range(total_steps))

    def __setitem__(self, t: int, step: TrajectoryStep) -> None:
        self.trajectory_continaer[t] = step

    def __getitem__(self, t: int) -> TrajectoryStep:
        if t == -1:
            t = self.total_steps
        return self.trajectory_continaer[t]

    def __len__(self):
        return len(self.trajectory_continaer)

    def __iter__(self):
        return iter(self.trajectory_continaer)

    def get_atoms(self, t: int = 0, idx: int = None):
        st = self[t]
        return step_to_atoms(st.atom_types, st.frac_coords, st.lattices, st.num_atoms, idx)

    def get_trajectory(self, idx: int = None):
        return [self.get_atoms(t, idx) for t in range(self.total_steps + 1)]


def step_to_atoms(atom_types, frac_coords, lattices, num_atoms, idx: int = None) -> Union[List, object]:
    """schema.py:57-83: split per crystal, clamp classes > 103 to 0, build
    Atoms(numbers, cell, pbc) with scaled positions, sort by symbol."""
    a = atom_types.detach().cpu()
    a = torch.where(a <= 103, a, 0).numpy()
    x = frac_coords.detach().cpu().numpy()
    lat = lattices.detach().cpu().numpy()
    nat = [int(n) for n in (num_atoms.tolist() if torch.is_tensor(num_atoms) else num_atoms)]
    out, off = [], 0
    for g, n in enumerate(nat):
        out.append(sort_atoms(make_atoms(a[off:off + n], lat[g], x[off:off + n])))
        off += n
    return out if idx is None else out[idx]
