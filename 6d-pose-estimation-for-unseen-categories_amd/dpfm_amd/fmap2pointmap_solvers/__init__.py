"""fmap -> point-map solvers (reference fmap2pointmap_solvers/__init__.py:1-8).

`choose_fmap2pointmap_solver(solver)` keeps the gin-configurable selector's contract
(config/dpfm_orig.gin:71 binds spacial_filtering_fmap2pointmap); without gin it simply
returns the solver it is given (default: the spatial-filtering solver)."""
from .naive import naive_fmap2pointmap, nn_query
from .spacial_filtering import spacial_filtering_fmap2pointmap, spacial_filtering


def choose_fmap2pointmap_solver(solver=None):
    return solver if solver is not None else spacial_filtering_fmap2pointmap
