"""Protocols of the reference's ``byzantinerandomizedconsensus.core`` package, backed by the
MI355X engine (``byzantinerandomizedconsensus_amd.network``)."""
