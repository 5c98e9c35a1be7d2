"""Drop-in replacements for the reference's ``modules`` package.

Put ``genetic-gaussian-splats_amd/`` ahead of the reference checkout on
``sys.path`` and ``from modules.render import render_splats_rgb_triton``,
``modules.fitness``, ``modules.algorithm``, ``modules.annealing`` … resolve to
the MI355X implementation.  Every other ``modules`` directory on ``sys.path``
(the reference's) is appended to this package's search path, so modules not
restated here — ``modules.config`` — still come from the reference checkout.
See INTEGRATION.md.
"""
from pkgutil import extend_path

__path__ = extend_path(__path__, __name__)
