"""``Consensus`` / ``IConsensusHandler`` (reference: base/consensus.py:4-24)."""
from abc import ABCMeta, abstractmethod


class Consensus(metaclass=ABCMeta):
    """A consensus protocol: ``propose`` starts an instance with a value."""

    @abstractmethod
    def propose(self, message):
        pass


class IConsensusHandler(metaclass=ABCMeta):
    """The DECIDE upcall of a consensus protocol."""

    @abstractmethod
    def decide(self, message):
        pass
