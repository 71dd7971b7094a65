"""A brb_test.py-style driver (the reference's test/brb_test.py shape): 4 nodes, f = 1, each
node SENDs one payload; the handler prints every delivery.  It imports only the reference's
module paths, so it runs unchanged on the reference or, with this repo on PYTHONPATH, on the
MI355X engine (the run happens at interpreter exit)."""
from byzantinerandomizedconsensus.base.broadcast import IBroadcastHandler
from byzantinerandomizedconsensus.core.brbroadcast import BRBroadcast


class Printer(IBroadcastHandler):
    def deliver(self, message):
        print(message)


N, f = 4, 1
addresses = [("localhost", 5000 + k) for k in range(N)]
replicas = [BRBroadcast(N, f, a, addresses, Printer()) for a in addresses]
for r in replicas:
    r.broadcast_listener()
for k, r in enumerate(replicas, start=1):
    r.broadcast(BRBroadcast.SEND, "TEST " + str(k))
