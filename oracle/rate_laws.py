"""Oracle (TEST INFRASTRUCTURE ONLY): convenience rate laws, evaluated the way
the reference evaluates them.

Restates vivarium/library/kinetic_rate_laws.py:
  * configuration with shared list objects ............ :43-98
  * in-place None-Km removal (aliasing) ................ :126-135
  * kcat selection / kcat_r NameError .................. :123-147
  * closure arithmetic (numerator, denominator) ........ :149-178
  * cofactor_numerator / cofactor_denominator .......... :100-104
  * get_fluxes (0.0 + sum over enzymes) ................ :277-297
Floating-point operation order follows the reference exactly (the products
over a cofactor list are sequential, as numpy.prod is for these sizes --
verified in tests/test_oracle.py).
"""

from __future__ import annotations


class OracleFluxModel:
    """Restatement of ``KineticFluxModel`` with lazily-read shared lists."""

    def __init__(self, reactions, kinetic_parameters):
        self.reactions = dict(reactions)
        self.kinetic_parameters = kinetic_parameters
        self.reaction_ids = list(kinetic_parameters.keys())

        # --- configuration (shared list objects) ---
        partition_of = {}
        cofactors_of = {}
        for rid, spec in self.reactions.items():
            for enz in spec['catalyzed by']:
                partition_of.setdefault(enz, [])
                cofactors_of.setdefault(enz, {})
        for rid, spec in self.reactions.items():
            st = spec.get('stoichiometry')
            own = [[m for m, c in st.items() if c < 0]]
            if spec.get('is reversible', False):
                own.append([m for m, c in st.items() if c > 0])
            for enz in spec.get('catalyzed by', None):
                rivals = []
                for other, spec2 in self.reactions.items():
                    if other != rid and enz in spec2['catalyzed by']:
                        rivals.append([m for m, c in spec2['stoichiometry'].items() if c < 0])
                partition_of[enz] = rivals + own
                cofactors_of[enz][rid] = own

        # --- rate laws (removal happens at construction; evaluation is lazy) ---
        self.laws = []  # (rid, enzyme, kcat, cofactor_sets, partition, params)
        for rid, spec in self.reactions.items():
            for enz in spec.get('catalyzed by'):
                if enz not in self.kinetic_parameters[rid]:
                    continue
                params = self.kinetic_parameters[rid][enz]
                sets = cofactors_of[enz][rid]
                part = partition_of[enz]
                for name, val in params.items():
                    if 'kcat' not in name and val is None:
                        for p in part:
                            if name in p:
                                p.remove(name)
                        for s in sets:
                            if name in s:
                                s.remove(name)
                if params.get('kcat_r'):
                    raise NameError("name 'cofactors' is not defined")
                self.laws.append((rid, enz, params.get('kcat_f'), sets, part, params))

    @staticmethod
    def _num_factor(c, km):
        return c / km if km else 0

    @staticmethod
    def _den_factor(c, km):
        return 1 + c / km if km else 1

    def rate_law_flux(self, law, conc):
        rid, enz, kcat, sets, part, params = law
        num = 0
        for s in sets:
            term = 1.0
            for m in s:
                term = term * self._num_factor(conc[m], params[m])
            num += kcat * term
        num *= conc[enz]
        den = 1
        for p in part:
            term = 1.0
            for m in p:
                term = term * self._den_factor(conc[m], params[m])
            den += term - 1
        return num / den

    def get_fluxes(self, conc):
        out = {rid: 0.0 for rid in self.reaction_ids}
        for law in self.laws:
            out[law[0]] += self.rate_law_flux(law, conc)
        return out
