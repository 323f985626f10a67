"""Structured brick mesh emitting the reference's DG face / node conventions.

Host-side setup (out of the timed path).  The reference builds its mesh with p4est
(p4est.c:1030-2043 -> mod_p4est.F90:216-415); p4est is not available here, so this
module emits an equivalent single-block brick with the conventions the hot path
relies on:

* DG node numbering ``I = (e-1)*P + (j-1)*ngl + i`` (``intma_dg``, mod_grid.F90:230-239)
  and quad numbering ``Iq = (e-1)*Q + (j-1)*nq + i`` (``intma_dg_quad``, :242-250).
* ``face(7,f)`` = left element, ``face(8,f)`` = right element (>0) or ``-bc`` for a
  physical boundary (p4est.c:1669); ``face(8,f) = 0`` marks a processor face.
* ``imapl(:,n,f)`` / ``imapr(:,n,f)`` = local (i,j,k) of face node ``n`` in the left /
  right element, both ordered along the same physical direction.
* normals point out of the left element; ``jac_face = w * |dx/dxi|`` on the face
  (create_normals.F90, create_normals_quad.F90:101-113).

Everything is returned 1-based where the reference is 1-based (element ids, local
indices) so the arrays can be handed to a Fortran host unchanged.  Arrays are numpy
arrays in Fortran (column-major) order with the reference's leading dimensions,
compacted where the reference carries a dead 2-D face index (``(:,n,1,f)``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class BrickMesh:
    nelx: int
    nely: int
    xdims: tuple
    ydims: tuple
    ngl: int
    nq: int
    x_boundary: tuple = (4, 4)   # west, east  (mod_input x_boundary)
    y_boundary: tuple = (4, 4)   # south, north

    def __post_init__(self):
        self.nelem = self.nelx * self.nely
        self.npts = self.ngl * self.ngl
        self.nqq = self.nq * self.nq
        self.npoin = self.nelem * self.npts
        self.npoin_q = self.nelem * self.nqq
        self.dx = (self.xdims[1] - self.xdims[0]) / self.nelx
        self.dy = (self.ydims[1] - self.ydims[0]) / self.nely
        self._build_faces()

    # ------------------------------------------------------------------ faces
    def _build_faces(self):
        nelx, nely, ngl, nq = self.nelx, self.nely, self.ngl, self.nq
        # x-normal faces (constant x), ordered iy-major; face node n runs along +y
        iy, ix = np.meshgrid(np.arange(nely), np.arange(nelx + 1), indexing="ij")
        iy, ix = iy.ravel(), ix.ravel()
        elv = np.where(ix == 0, ix + iy * nelx + 1, ix - 1 + iy * nelx + 1)
        erv = np.where(ix == 0, -self.x_boundary[0],
                       np.where(ix == nelx, -self.x_boundary[1], ix + iy * nelx + 1))
        slv = np.where(ix == 0, 0, 1)                 # left side: 0=W 1=E 2=S 3=N
        srv = np.where((ix == 0) | (ix == nelx), -1, 0)
        # y-normal faces (constant y), ordered iy-major; face node n runs along +x
        jy, jx = np.meshgrid(np.arange(nely + 1), np.arange(nelx), indexing="ij")
        jy, jx = jy.ravel(), jx.ravel()
        elh = np.where(jy == 0, jx + 1, jx + (jy - 1) * nelx + 1)
        erh = np.where(jy == 0, -self.y_boundary[0],
                       np.where(jy == nely, -self.y_boundary[1], jx + jy * nelx + 1))
        slh = np.where(jy == 0, 2, 3)
        srh = np.where((jy == 0) | (jy == nely), -1, 2)
        el = np.concatenate([elv, elh]); er = np.concatenate([erv, erh])
        sl = np.concatenate([slv, slh]); sr = np.concatenate([srv, srh])
        nface = el.size
        self.nface = nface
        # NUMA local face ids (face(5:6)) of a 2-D mesh in the xy plane: p4est faces x-, x+, y-, y+
        # -> transform {4,5,2,3} + 1 (p4est.c:1551-1574, ORIENT = 2 when nglx, ngly > 1,
        # mod_p4est.F90:263-271), i.e. ksi = -/+1 -> 5/6, eta = -/+1 -> 3/4; the set-up routines
        # loop over face points by them (mod_grid_get_face_nq, mod_grid.F90:475-491)
        lid = np.array([5, 6, 3, 4], dtype=np.int32)
        face = np.zeros((8, nface), dtype=np.int32, order="F")
        face[4] = lid[sl]
        face[5] = np.where(sr >= 0, lid[np.maximum(sr, 0)], 0)
        face[6] = el
        face[7] = er
        self.face = face

        def local_ij(side, m):
            # 1-based (i,j) of the n-th of m points on each side; returns (nface, m)
            n = np.arange(1, m + 1)[None, :]
            s = side[:, None]
            i = np.where(s == 0, 1, np.where(s == 1, m, n))
            j = np.where(s == 2, 1, np.where(s == 3, m, n))
            i = np.where(s < 0, 0, i)
            j = np.where(s < 0, 0, j)
            return np.broadcast_to(i, (side.size, m)), np.broadcast_to(j, (side.size, m))

        def imap(side, m):
            i, j = local_ij(side, m)
            out = np.zeros((3, m, nface), dtype=np.int32, order="F")
            out[0] = i.T
            out[1] = j.T
            out[2] = np.where(side[None, :] < 0, 0, 1)
            return out

        self.imapl, self.imapr = imap(sl, ngl), imap(sr, ngl)
        self.imapl_q, self.imapr_q = imap(sl, nq), imap(sr, nq)
        onx = np.array([-1.0, 1.0, 0.0, 0.0])[sl]
        ony = np.array([0.0, 0.0, -1.0, 1.0])[sl]
        nv = np.zeros((3, ngl, nface), order="F")
        nv[0] = onx[None, :]
        nv[1] = ony[None, :]
        nvq = np.zeros((3, nq, nface), order="F")
        nvq[0] = onx[None, :]
        nvq[1] = ony[None, :]
        self.normal_vector, self.normal_vector_q = nv, nvq
        self._face_length = np.where(sl < 2, self.dy, self.dx)

    def finalize_face_jacobians(self, wgl, wnq):
        """jac_face = w * |d x/d s| with |d x/d s| = length/2 (create_normals_quad.F90:101-113)."""
        half = 0.5 * self._face_length
        self.jac_face = np.asfortranarray(wgl[:, None] * half[None, :])
        self.jac_faceq = np.asfortranarray(wnq[:, None] * half[None, :])

    # ------------------------------------------------------------ coordinates
    def node_coords(self, xgl):
        """coord(1:2, npoin) of the DG nodes (element-major, i fastest)."""
        ngl = self.ngl
        e = np.arange(self.nelem)
        ex = e % self.nelx
        ey = e // self.nelx
        xi = (xgl + 1.0) * 0.5
        x = self.xdims[0] + (ex[:, None, None] + xi[None, None, :]) * self.dx
        y = self.ydims[0] + (ey[:, None, None] + xi[None, :, None]) * self.dy
        x = np.broadcast_to(x, (self.nelem, ngl, ngl))
        y = np.broadcast_to(y, (self.nelem, ngl, ngl))
        coord = np.zeros((3, self.npoin), order="F")
        coord[0] = x.reshape(-1)
        coord[1] = y.reshape(-1)
        return coord

    def face_neighbors(self):
        """For each element, its 4 faces (W,E,S,N) as 0-based face ids and whether
        the element is the left (0) or right (1) side of that face."""
        nelx, nely = self.nelx, self.nely
        nvert = nely * (nelx + 1)
        e = np.arange(self.nelem)
        ex, ey = e % nelx, e // nelx
        fW = ey * (nelx + 1) + ex
        fE = fW + 1
        fS = nvert + ey * nelx + ex
        fN = fS + nelx
        faces = np.stack([fW, fE, fS, fN], axis=1).astype(np.int32)
        side = np.zeros_like(faces)
        side[:, 0] = np.where(ex == 0, 0, 1)   # west face: element is right unless boundary
        side[:, 1] = 0
        side[:, 2] = np.where(ey == 0, 0, 1)
        side[:, 3] = 0
        return faces, side
