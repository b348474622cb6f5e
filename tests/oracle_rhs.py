"""Test-side import of the oracle-backed RHS objects (oracle/oracle_rhs.py)."""
from oracle.oracle_rhs import OracleChainRHS, OracleFKRHS  # noqa: F401
