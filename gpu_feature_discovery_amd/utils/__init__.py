"""Support code for tests, benchmarks and builds (not used by the daemon).

* :mod:`.synth` - synthetic KFD/DRM/PCI sysfs trees (1-8 GPUs, SPX..CPX,
  NPS1..NPS4, SR-IOV PF/VF, passthrough) with random device identities,
* :mod:`.golden` - byte goldens and bidirectional regex goldens,
* :mod:`.build` - in-tree build of the native targets,
* :mod:`.proc` - process wall time without subprocess's polling wait.
"""
