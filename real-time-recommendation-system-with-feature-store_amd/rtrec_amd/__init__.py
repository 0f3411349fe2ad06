"""MI355X-native two-tower retrieval path: a drop-in for the reference's
``src.models`` / ``src.serving`` / ``src.training`` surface under the
non-colliding package name ``rtrec_amd`` (so it imports beside the reference's
own ``src`` package).

Compute runs only through librtrec_hip.so (see ``rtrec_amd.native``)."""
