"""MI355X-native two-tower retrieval path (drop-in for the reference's
``src.models`` / ``src.serving`` / ``src.training`` surface).

Compute runs only through librtrec_hip.so (see ``src.native``)."""
