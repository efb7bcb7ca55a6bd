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


# ---------------------------------------------------------------------------------------------
# CIF output (the reference's scripts convert the sampled ase.Atoms with pymatgen's
# AseAtomsAdaptor and write `gen_{i}.cif`, chemeleon/scripts/sample_prompt.py:38-42; neither
# pymatgen nor ase is needed here): P1 cell + fractional coordinates + symbols.
# ---------------------------------------------------------------------------------------------
def cell_parameters(cell) -> tuple:
    """(a, b, c, alpha, beta, gamma) in Angstrom / degrees of a row-vector cell [3, 3]."""
    v = np.asarray(cell, dtype=np.float64).reshape(3, 3)
    lens = np.linalg.norm(v, axis=1)

    def ang(i, j):
        d = lens[i] * lens[j]
        return 90.0 if d == 0 else float(np.degrees(np.arccos(np.clip(np.dot(v[i], v[j]) / d, -1.0, 1.0))))

    return float(lens[0]), float(lens[1]), float(lens[2]), ang(1, 2), ang(0, 2), ang(0, 1)


def _formula_counts(symbols):
    counts: Dict[str, int] = OrderedDict()
    for s in symbols:
        counts[s] = counts.get(s, 0) + 1
    return counts


def atoms_to_cif(atoms, name: Optional[str] = None) -> str:
    """One structure (ase.Atoms or this module's Atoms) as a P1 CIF document."""
    symbols = list(atoms.get_chemical_symbols())
    frac = np.asarray(atoms.get_scaled_positions(), dtype=np.float64).reshape(-1, 3)
    a, b, c, al, be, ga = cell_parameters(np.asarray(atoms.cell))
    vol = float(abs(np.linalg.det(np.asarray(atoms.cell, dtype=np.float64).reshape(3, 3))))
    counts = _formula_counts(sorted(symbols))
    formula_sum = " ".join(f"{s}{n}" for s, n in counts.items())
    name = name or "".join(f"{s}{n}" for s, n in counts.items())
    lines = [
        f"data_{name}",
        "_symmetry_space_group_name_H-M   'P 1'",
        f"_cell_length_a   {a:.8f}",
        f"_cell_length_b   {b:.8f}",
        f"_cell_length_c   {c:.8f}",
        f"_cell_angle_alpha   {al:.8f}",
        f"_cell_angle_beta   {be:.8f}",
        f"_cell_angle_gamma   {ga:.8f}",
        "_symmetry_Int_Tables_number   1",
        f"_chemical_formula_structural   {name}",
        f"_chemical_formula_sum   '{formula_sum}'",
        f"_cell_volume   {vol:.8f}",
        "_cell_formula_units_Z   1",
        "loop_",
        " _symmetry_equiv_pos_site_id",
        " _symmetry_equiv_pos_as_xyz",
        "  1  'x, y, z'",
        "loop_",
        " _atom_site_type_symbol",
        " _atom_site_label",
        " _atom_site_symmetry_multiplicity",
        " _atom_site_fract_x",
        " _atom_site_fract_y",
        " _atom_site_fract_z",
        " _atom_site_occupancy",
    ]
    seen: Dict[str, int] = {}
    for s, (x, y, z) in zip(symbols, frac):
        k = seen.get(s, 0)
        seen[s] = k + 1
        lines.append(f"  {s}  {s}{k}  1  {x:.8f}  {y:.8f}  {z:.8f}  1")
    return "\n".join(lines) + "\n"


def write_cif(atoms, path) -> str:
    """Writes one structure to `path` (a .cif file); returns the path."""
    path = str(path)
    with open(path, "w") as f:
        f.write(atoms_to_cif(atoms))
    return path


def save_structures(atoms_list, save_dir, prefix: str = "gen_") -> List[str]:
    """The reference's output step (sample_prompt.py:38-42): `save_dir/gen_{i}.cif` per structure."""
    import os
    os.makedirs(str(save_dir), exist_ok=True)
    return [write_cif(at, os.path.join(str(save_dir), f"{prefix}{i}.cif")) for i, at in enumerate(atoms_list)]
