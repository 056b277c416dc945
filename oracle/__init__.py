"""CPU oracle for the LoadBalancerK8sEnv hot path — TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
