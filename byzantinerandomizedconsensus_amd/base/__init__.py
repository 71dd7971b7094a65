"""Interfaces of the reference's ``byzantinerandomizedconsensus.base`` package."""
