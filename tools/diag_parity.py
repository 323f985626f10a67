import sys, numpy as np
sys.path[:0]=['h-numo_amd','oracle','tests']
import oracle as O
from hnumo.case import build_case, make_config
from hnumo.engine import Engine
from util import rel
for cfg in ['bump10','dg25L3']:
    c=build_case(make_config(cfg)); o=O.Oracle(c); e=Engine(c)
    q,qb,qp=o.state(); qe,qbe,qpe=e.state()
    o.btp_bcl_coeffs(qp); e.btp_bcl_coeffs(qp)
    r_o=o.create_rhs_btp(qb,qp); r_e=e.create_rhs_btp(qb,qp)
    print(cfg,'rhs0', [rel(r_e[v],r_o[v]) for v in range(3)])
    o.ti_barotropic_ssprk(qb,qp); e.ti_barotropic_ssprk(qbe,qp)
    print(cfg,'subcycle qb', [rel(qbe[v],qb[v]) for v in range(4)])
    q,qb,qp=o.state(); qe,qbe,qpe=e.state()
    for s in range(2):
        o.ti_rk_bcl(q,qb,qp); e.ti_rk_bcl(qe,qbe,qpe)
        print(cfg,'step',s+1,'qb',[rel(qbe[v],qb[v]) for v in range(4)], 'q', [rel(qe[v],q[v]) for v in range(3)], 'qp', [rel(qpe[v],qp[v]) for v in range(3)])
