"""Structure output: the sorted Atoms of step_to_atoms and the CIF files
the reference's scripts write (chemeleon/scripts/sample_prompt.py:38-42: pymatgen Structure ->
gen_{i}.cif), produced here without pymatgen / ase. CPU only."""

import numpy as np
import torch

from chemeleon_amd.modules.schema import atoms_to_cif, cell_parameters, save_structures, step_to_atoms


def parse_cif(text):
    """Minimal P1 CIF reader: cell parameters and (symbol, frac) sites."""
    vals, sites, in_sites, cols = {}, [], False, []
    for line in text.splitlines():
        t = line.split()
        if not t:
            continue
        if t[0].startswith("_cell_length") or t[0].startswith("_cell_angle"):
            vals[t[0]] = float(t[1])
        elif t[0] == "loop_":
            in_sites, cols = False, []
        elif t[0].startswith("_atom_site"):
            in_sites = True
            cols.append(t[0])
        elif in_sites and len(t) == len(cols):
            row = dict(zip(cols, t))
            sites.append((row["_atom_site_type_symbol"],
                          [float(row[f"_atom_site_fract_{c}"]) for c in "xyz"]))
    return vals, sites


def lattice_from_parameters(a, b, c, al, be, ga):
    al, be, ga = np.radians([al, be, ga])
    v1 = [a, 0, 0]
    v2 = [b * np.cos(ga), b * np.sin(ga), 0]
    cx = c * np.cos(be)
    cy = c * (np.cos(al) - np.cos(be) * np.cos(ga)) / np.sin(ga)
    return np.array([v1, v2, [cx, cy, np.sqrt(c * c - cx * cx - cy * cy)]])


def test_cif_round_trip(tmp_path):
    g = torch.Generator().manual_seed(4)
    nat = [3, 5]
    a = torch.tensor([8, 22, 22, 3, 25, 8, 8, 8])
    x = torch.rand(8, 3, generator=g)
    lat = torch.randn(2, 3, 3, generator=g) + 4 * torch.eye(3)
    structs = step_to_atoms(a, x, lat, nat)
    paths = save_structures(structs, tmp_path / "out")
    assert [p.split("/")[-1] for p in paths] == ["gen_0.cif", "gen_1.cif"]
    for s, p, L in zip(structs, paths, lat.numpy()):
        vals, sites = parse_cif(open(p).read())
        par = [vals[k] for k in ("_cell_length_a", "_cell_length_b", "_cell_length_c", "_cell_angle_alpha",
                                 "_cell_angle_beta", "_cell_angle_gamma")]
        np.testing.assert_allclose(par, cell_parameters(L), rtol=1e-7)
        # same metric (cell up to a rotation)
        Lr = lattice_from_parameters(*par)
        np.testing.assert_allclose(Lr @ Lr.T, L.astype(np.float64) @ L.T.astype(np.float64), rtol=1e-6, atol=1e-6)
        assert [sy for sy, _ in sites] == s.get_chemical_symbols()
        np.testing.assert_allclose([f for _, f in sites], s.get_scaled_positions(), atol=1e-8)
    # sorted by symbol, as ase.build.tools.sort
    assert structs[1].get_chemical_symbols() == ["Li", "Mn", "O", "O", "O"]
    assert "_symmetry_space_group_name_H-M   'P 1'" in atoms_to_cif(structs[0])
