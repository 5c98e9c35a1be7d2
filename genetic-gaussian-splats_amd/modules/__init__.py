"""Drop-in replacements for the reference's hot-path modules.

Put ``genetic-gaussian-splats_amd/`` ahead of the reference checkout on
``sys.path`` (or copy ``modules/render.py``, ``modules/fitness.py`` and
``modules/encode.py`` over the reference's) and ``from modules.render import
render_splats_rgb_triton`` / ``from modules.fitness import fitness_population``
resolve to the MI355X implementation.  See INTEGRATION.md.
"""
