"""float64 reference kinematics for articulations (test helper).

Independent of the engine's spatial-algebra code: forward kinematics by
composing joint transforms, geometric Jacobians, and the joint-space mass matrix
as sum_l (m_l Jv_l^T Jv_l + Jw_l^T I_l Jw_l) over link COM Jacobians — the
textbook definition, not CRBA. Reads the packed model arrays of
test_isaacgym_amd._sim.Sim.build_model (mg_model layout, include/migym.h).
"""
import numpy as np


def qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def qmat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


class Articulation:
    """One articulation template of a packed model."""

    def __init__(self, A, tmpl=0):
        ti = A["artic_tmpl_i"][tmpl]
        fl, self.L, self.D = int(ti[0]), int(ti[1]), int(ti[2])
        self.lf = A["tmpl_link_f"][fl:fl + self.L].astype(np.float64)
        self.li = A["tmpl_link_i"][fl:fl + self.L]
        self.A = A

    def fk(self, base_pose, q):
        """World (position, rotation matrix, joint axis) of every link frame."""
        ps = [np.asarray(base_pose[0:3], np.float64)]
        qb = np.asarray(base_pose[3:7], np.float64)
        qs = [qb / np.linalg.norm(qb)]
        zs = [np.zeros(3)]
        for l in range(1, self.L):
            p, jt, d = int(self.li[l, 0]), int(self.li[l, 1]), int(self.li[l, 2])
            po, qo, ax = self.lf[l, 0:3], self.lf[l, 3:7], self.lf[l, 7:10]
            qrel, rr = qo.copy(), po.copy()
            ball = int(round(self.lf[l, 10]))
            if ball == 1:           # ball joint: exp of the rotation vector q[d..d+2]
                th = np.asarray(q[d:d + 3], np.float64)
                t = np.linalg.norm(th)
                if t > 0:
                    qrel = qmul(qo, np.array([*(th / t * np.sin(0.5 * t)), np.cos(0.5 * t)]))
            elif ball > 1:          # its later links: no turn of their own
                pass
            elif jt == 1:
                s, c = np.sin(0.5 * q[d]), np.cos(0.5 * q[d])
                qrel = qmul(qo, np.array([ax[0] * s, ax[1] * s, ax[2] * s, c]))
            elif jt == 2:
                rr = po + qmat(qo) @ (ax * q[d])
            ql = qmul(qs[p], qrel)
            ql /= np.linalg.norm(ql)
            ps.append(ps[p] + qmat(qs[p]) @ rr)
            qs.append(ql)
            zs.append(qmat(ql) @ ax)
        return ps, [qmat(x) for x in qs], zs

    def point_jacobian(self, ps, zs, l, pt):
        """(6, D) Jacobian of world point pt fixed to link l: [linear; angular]."""
        J = np.zeros((6, self.D))
        j = l
        while j > 0:
            jt, d = int(self.li[j, 1]), int(self.li[j, 2])
            if d >= 0:
                if jt == 1:
                    J[0:3, d] = np.cross(zs[j], pt - ps[j])
                    J[3:6, d] = zs[j]
                else:
                    J[0:3, d] = zs[j]
            j = int(self.li[j, 0])
        return J

    def bodies(self):
        """(link, local body) of the real links (a ball joint's two virtual
        links have body -1: no Jacobian row, no mass)."""
        return [(l, int(self.li[l, 3])) for l in range(self.L) if int(self.li[l, 3]) >= 0]

    def jacobian(self, base_pose, q):
        """(B-1, 6, D): body origins, as mg_refresh_jacobian."""
        ps, Rs, zs = self.fk(base_pose, q)
        return np.stack([self.point_jacobian(ps, zs, l, ps[l]) for l, _ in self.bodies()[1:]])

    def mass_matrix(self, base_pose, q, first_body):
        """(D, D) joint-space inertia (no armature)."""
        ps, Rs, zs = self.fk(base_pose, q)
        M = np.zeros((self.D, self.D))
        for l, b in self.bodies()[1:]:
            mrow = self.A["body_mass"][first_body + b].astype(np.float64)
            m, com, iq, invI = mrow[11], mrow[8:11], mrow[4:8], mrow[1:4]
            Ip = np.diag([1.0 / x if x > 0 else 0.0 for x in invI])
            Rl = Rs[l] @ qmat(iq)
            Iw = Rl @ Ip @ Rl.T
            J = self.point_jacobian(ps, zs, l, ps[l] + Rs[l] @ com)
            M += m * J[0:3].T @ J[0:3] + J[3:6].T @ Iw @ J[3:6]
        return M


    # ---- floating base: 6 root columns first — root linear velocity of the
    # base-link origin x0 (world xyz), then root angular velocity (world xyz) —
    # then the DOFs (the layout of mg_refresh_jacobian for a floating base)
    def point_jacobian_fb(self, ps, zs, l, pt):
        """(6, 6 + D) Jacobian of world point pt fixed to link l."""
        J = np.zeros((6, 6 + self.D))
        J[0:3, 0:3] = np.eye(3)
        r = pt - ps[0]
        for k in range(3):
            e = np.eye(3)[k]
            J[0:3, 3 + k] = np.cross(e, r)
            J[3:6, 3 + k] = e
        J[:, 6:] = self.point_jacobian(ps, zs, l, pt)
        return J

    def jacobian_fb(self, base_pose, q):
        """(L, 6, 6 + D): every link origin, the root link included."""
        ps, Rs, zs = self.fk(base_pose, q)
        return np.stack([self.point_jacobian_fb(ps, zs, l, ps[l]) for l, _ in self.bodies()])

    def mass_matrix_fb(self, base_pose, q, first_body):
        """(6 + D, 6 + D) inertia in the same generalized velocities (no armature)."""
        ps, Rs, zs = self.fk(base_pose, q)
        M = np.zeros((6 + self.D, 6 + self.D))
        for l, b in self.bodies():
            mrow = self.A["body_mass"][first_body + b].astype(np.float64)
            m, com, iq, invI = mrow[11], mrow[8:11], mrow[4:8], mrow[1:4]
            Ip = np.diag([1.0 / x if x > 0 else 0.0 for x in invI])
            Rl = Rs[l] @ qmat(iq)
            Iw = Rl @ Ip @ Rl.T
            J = self.point_jacobian_fb(ps, zs, l, ps[l] + Rs[l] @ com)
            M += m * J[0:3].T @ J[0:3] + J[3:6].T @ Iw @ J[3:6]
        return M
