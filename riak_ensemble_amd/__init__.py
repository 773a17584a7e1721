"""riak_ensemble_amd — MI355X-native synctree hashing & exchange path.

The product is ``libsynctree_hip.so`` (HIP kernels for gfx950 behind the C-ABI
in include/synctree_hip.h) plus ``riak_ensemble_amd.synctree``, a host-side
mirror of the reference's ``synctree`` module API that calls it.
"""
__all__ = ['synctree', 'synctree_hip', 'workload']
