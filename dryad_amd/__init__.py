"""Dryad-AMD: an MI355X-native DAG data-parallel engine with the DryadLINQ programming model.

Public API (reference LinqToDryad): ``DryadLinqContext`` + lazy ``Query`` operators, ``LineRecord``,
``Pair``, ``ForkTuple``/``ForkValue``, attributes (``homomorphic``, ``decomposable``, ...), and
``DryadLinqJobInfo``.
"""
__version__ = "0.1.0"

from .errors import DryadLinqException, ErrorCode  # noqa: E402,F401
from .types import (LineRecord, Pair, ForkTuple, ForkValue, SqlDateTime)  # noqa: E402,F401
from . import types  # noqa: E402,F401
from .attributes import (homomorphic, resource, decomposable, associative, custom_serializer,  # noqa: E402,F401
                         IDecomposable, IAssociative)
from .context import (DryadLinqContext, PlatformKind, ExecutorKind, CompressionScheme,  # noqa: E402,F401
                      QueryLoggingLevel, LocalCpuCluster, LocalGpuNode, DryadLinqCluster)
from .query import Query, MultiQuery, KeyedMultiQuery  # noqa: E402,F401
from .jobinfo import DryadLinqJobInfo, JobStatus  # noqa: E402,F401
from .enumerable import Grouping  # noqa: E402,F401
