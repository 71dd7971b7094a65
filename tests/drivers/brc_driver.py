"""A brc_test.py-style driver (the reference's test/brc_test.py shape): 6 nodes, f = 1, every
node proposes 3; the handler prints every decision.  Reference module paths only."""
from byzantinerandomizedconsensus.base.consensus import IConsensusHandler
from byzantinerandomizedconsensus.core.byzantinerandomizedconsensus import ByzantineRandomizedConsensus


class Printer(IConsensusHandler):
    def decide(self, message):
        print("Consensus protocol decided on message: " + message)


N, f = 6, 1
addresses = [("localhost", 5555 + k) for k in range(N)]
replicas = [ByzantineRandomizedConsensus(N, f, addresses, a, Printer()) for a in addresses]
for r in replicas:
    r.message_queue.put_nowait(3)
    r.start()
