"""`perwez` -> reth_amd.perwez (perwez/perwez/__init__.py:18-32, client/socket.py:19-122)"""
from reth_amd.perwez import RecvSocket, SendSocket, start_server  # noqa: F401
