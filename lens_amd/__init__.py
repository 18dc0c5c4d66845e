"""lens_amd -- MI355X-native batched agent-kinetics engine for Vivarium-style colonies.

Host side of the drop-in boundary (reference: CovertLab/Lens ``vivarium``):

* :mod:`lens_amd.rate_law_compiler` -- reaction dicts -> flat SoA table
* :mod:`lens_amd.native`            -- ctypes binding of ``include/vk_kinetics.h``
* :mod:`lens_amd.process`           -- ``BatchedConvenienceKinetics`` (Process API)
* :mod:`lens_amd.invoke`            -- ``BatchedInvoke`` for ``Experiment(config['invoke'])``
* :mod:`lens_amd.colony`            -- persistent SoA colony + lattice engine
"""

__version__ = '0.1.0'
