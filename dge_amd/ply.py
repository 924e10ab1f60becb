"""PLY vertex I/O for Gaussian scenes.

The reference reads and writes its scenes with the third-party ``plyfile``
package (gaussian_model.py:410-445 save_ply, :455-551 load_ply), which is not
installed here.  This module restates the part of the PLY format those calls
use — one ``vertex`` element of scalar properties, ``binary_little_endian``
(what ``PlyData([el]).write`` emits) or ``ascii`` / ``binary_big_endian`` on
read — with numpy structured arrays, so files written by either side load in
the other.  Property order on write is the reference's
``construct_list_of_attributes`` (x, y, z, nx, ny, nz, f_dc_*, f_rest_*,
opacity, scale_*, rot_*), all float32.
"""
from __future__ import annotations

import numpy as np

_PLY_TYPES = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1",
    "short": "i2", "int16": "i2", "ushort": "u2", "uint16": "u2",
    "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}
_NP_TO_PLY = {"i1": "char", "u1": "uchar", "i2": "short", "u2": "ushort", "i4": "int", "u4": "uint",
              "f4": "float", "f8": "double"}


class PlyError(ValueError):
    pass


def read_ply(path):
    """-> {element name: numpy structured array} for a PLY file of scalar properties."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise PlyError(f"{path}: not a PLY file")
        fmt, elements = None, []
        while True:
            line = f.readline()
            if not line:
                raise PlyError(f"{path}: header without end_header")
            tok = line.decode("ascii", "replace").split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                elements.append((tok[1], int(tok[2]), []))
            elif tok[0] == "property":
                if not elements:
                    raise PlyError(f"{path}: property before element")
                if tok[1] == "list":
                    raise PlyError(f"{path}: list properties are not supported ({tok[-1]})")
                if tok[1] not in _PLY_TYPES:
                    raise PlyError(f"{path}: unknown property type {tok[1]}")
                elements[-1][2].append((tok[2], _PLY_TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        out = {}
        if fmt == "ascii":
            for name, count, props in elements:
                dt = np.dtype([(n, t) for n, t in props])
                rows = [f.readline().split() for _ in range(count)]
                arr = np.empty(count, dtype=dt)
                for j, (n, t) in enumerate(props):
                    arr[n] = np.array([r[j] for r in rows], dtype=t) if count else np.empty(0, t)
                out[name] = arr
        elif fmt in ("binary_little_endian", "binary_big_endian"):
            order = "<" if fmt == "binary_little_endian" else ">"
            for name, count, props in elements:
                dt = np.dtype([(n, order + t) for n, t in props])
                buf = f.read(dt.itemsize * count)
                if len(buf) != dt.itemsize * count:
                    raise PlyError(f"{path}: truncated element {name}")
                out[name] = np.frombuffer(buf, dtype=dt).astype(dt.newbyteorder("="))
        else:
            raise PlyError(f"{path}: unsupported format {fmt}")
    return out


def write_ply(path, vertex: np.ndarray) -> None:
    """Write one ``vertex`` element (numpy structured array) as binary_little_endian."""
    props = []
    for n in vertex.dtype.names:
        t = vertex.dtype[n].str.lstrip("<>=|")
        if t not in _NP_TO_PLY:
            raise PlyError(f"unsupported dtype {vertex.dtype[n]} for property {n}")
        props.append((n, t))
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {len(vertex)}"]
    header += [f"property {_NP_TO_PLY[t]} {n}" for n, t in props]
    header += ["end_header"]
    le = np.dtype([(n, "<" + t) for n, t in props])
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(np.ascontiguousarray(vertex.astype(le)).tobytes())


def attribute_names(n_dc: int, n_rest: int, n_scale: int = 3, n_rot: int = 4):
    """gaussian_model.py:396-408 construct_list_of_attributes."""
    names = ["x", "y", "z", "nx", "ny", "nz"]
    names += [f"f_dc_{i}" for i in range(n_dc)]
    names += [f"f_rest_{i}" for i in range(n_rest)]
    names += ["opacity"]
    names += [f"scale_{i}" for i in range(n_scale)]
    names += [f"rot_{i}" for i in range(n_rot)]
    return names


def gaussians_to_vertex(xyz, f_dc, f_rest, opacity, scaling, rotation) -> np.ndarray:
    """Raw parameters (numpy, [P,3] / [P,1,3] / [P,M-1,3] / [P,1] / [P,3] / [P,4]) -> vertex array
    laid out as save_ply does: features transposed to channel-major and flattened (:410-445)."""
    P = xyz.shape[0]
    fdc = np.ascontiguousarray(np.transpose(f_dc, (0, 2, 1)).reshape(P, -1))
    frest = np.ascontiguousarray(np.transpose(f_rest, (0, 2, 1)).reshape(P, -1))
    cols = [xyz, np.zeros_like(xyz), fdc, frest, opacity.reshape(P, 1), scaling, rotation]
    attrs = np.concatenate([c.astype(np.float32).reshape(P, -1) for c in cols], axis=1)
    names = attribute_names(fdc.shape[1], frest.shape[1], scaling.shape[1], rotation.shape[1])
    v = np.empty(P, dtype=[(n, "f4") for n in names])
    for j, n in enumerate(names):
        v[n] = attrs[:, j]
    return v


def vertex_to_gaussians(v: np.ndarray):
    """Vertex array -> (xyz [P,3], f_dc [P,1,3], f_rest [P,M-1,3], opacity [P,1], scaling [P,S],
    rotation [P,R], max_sh_degree) as load_ply builds them (:455-551): f_rest_* and scale_*/rot_*
    sorted by their numeric suffix, features reshaped channel-major then transposed."""
    names = v.dtype.names
    P = len(v)
    xyz = np.stack([v["x"], v["y"], v["z"]], axis=1).astype(np.float32)
    opacity = np.asarray(v["opacity"], dtype=np.float32)[:, None]
    f_dc = np.zeros((P, 3, 1), dtype=np.float32)
    for c in range(3):
        f_dc[:, c, 0] = v[f"f_dc_{c}"]

    def suffixed(prefix):
        return sorted((n for n in names if n.startswith(prefix)), key=lambda x: int(x.split("_")[-1]))

    rest = suffixed("f_rest_")
    max_sh_degree = int(((len(rest) + 3) / 3) ** 0.5 - 1)
    f_rest = np.zeros((P, len(rest)), dtype=np.float32)
    for i, n in enumerate(rest):
        f_rest[:, i] = v[n]
    f_rest = f_rest.reshape(P, 3, (max_sh_degree + 1) ** 2 - 1)
    scaling = np.stack([v[n] for n in suffixed("scale_")], axis=1).astype(np.float32)
    rotation = np.stack([v[n] for n in suffixed("rot")], axis=1).astype(np.float32)
    return (xyz, np.ascontiguousarray(f_dc.transpose(0, 2, 1)), np.ascontiguousarray(f_rest.transpose(0, 2, 1)),
            opacity, scaling, rotation, max_sh_degree)
