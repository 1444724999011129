"""DryadLINQ-compatible exception hierarchy and error codes.

Error codes keep the reference's numbering (category base + offset) so that tooling keyed on
``DryadLinqException.ErrorCode`` keeps working (reference: LinqToDryad/DryadLinqFaultCodes.cs:30-278,
148 codes in 8 categories).  The table is data: ``ErrorCode.<Name>`` is the integer code.
"""
from __future__ import annotations

CATEGORY_BASE = {
    "QueryAPI": 0x01000000,
    "CodeGen": 0x02000000,
    "JobSubmission": 0x03000000,
    "Serialization": 0x04000000,
    "StoreClient": 0x05000000,
    "VertexRuntime": 0x06000000,
    "LocalDebug": 0x07000000,
    "Unknown": 0x0F000000,
}

_TABLE = {
    'TypeRequiredToBePublic': ('CodeGen', 0),
    'CustomSerializerMustSupportDefaultCtor': ('CodeGen', 1),
    'CustomSerializerMustBeClassOrStruct': ('CodeGen', 2),
    'TypeNotSerializable': ('CodeGen', 3),
    'CannotHandleSubtypes': ('CodeGen', 4),
    'UDTMustBeConcreteType': ('CodeGen', 5),
    'UDTHasFieldOfNonPublicType': ('CodeGen', 6),
    'UDTIsDelegateType': ('CodeGen', 7),
    'FailedToBuild': ('CodeGen', 8),
    'OutputTypeCannotBeAnonymous': ('CodeGen', 9),
    'InputTypeCannotBeAnonymous': ('CodeGen', 10),
    'BranchOfForkNotUsed': ('CodeGen', 11),
    'ComparerMustBeSpecifiedOrKeyTypeMustBeIComparable': ('CodeGen', 12),
    'ComparerMustBeSpecifiedOrKeyTypeMustBeIEquatable': ('CodeGen', 13),
    'ComparerExpressionMustBeSpecifiedOrElementTypeMustBeIEquatable': ('CodeGen', 14),
    'TooManyHomomorphicAttributes': ('CodeGen', 15),
    'HomomorphicApplyNeedsSamePartitionCount': ('CodeGen', 16),
    'UnrecognizedDataSource': ('CodeGen', 17),
    'CannotConcatDatasetsWithDifferentCompression': ('CodeGen', 21),
    'AggregateOperatorNotSupported': ('CodeGen', 23),
    'FinalizerReturnTypeMismatch': ('CodeGen', 24),
    'CannotHandleCircularTypes': ('CodeGen', 26),
    'OperatorNotSupported': ('CodeGen', 27),
    'AggregationOperatorRequiresIComparable': ('CodeGen', 28),
    'DecomposerTypeDoesNotImplementInterface': ('CodeGen', 29),
    'DecomposerTypeImplementsTooManyInterfaces': ('CodeGen', 30),
    'DecomposerTypesDoNotMatch': ('CodeGen', 31),
    'DecomposerTypeMustBePublic': ('CodeGen', 32),
    'DecomposerTypeDoesNotHavePublicDefaultCtor': ('CodeGen', 33),
    'AssociativeMethodHasWrongForm': ('QueryAPI', 34),
    'AssociativeTypeDoesNotImplementInterface': ('CodeGen', 35),
    'AssociativeTypeImplementsTooManyInterfaces': ('CodeGen', 36),
    'AssociativeTypesDoNotMatch': ('CodeGen', 37),
    'AssociativeTypeMustBePublic': ('CodeGen', 38),
    'AssociativeTypeDoesNotHavePublicDefaultCtor': ('CodeGen', 39),
    'CannotCreatePartitionNodeRandom': ('CodeGen', 43),
    'PartitionKeysNotProvided': ('CodeGen', 44),
    'PartitionKeysAreNotConsistentlyOrdered': ('CodeGen', 45),
    'IsDescendingIsInconsistent': ('CodeGen', 46),
    'BadSeparatorCount': ('CodeGen', 65),
    'TypeMustHaveDataMembers': ('CodeGen', 66),
    'CannotHandleObjectFields': ('CodeGen', 67),
    'CannotHandleDerivedtypes': ('CodeGen', 68),
    'MultipleOutputsWithSameDscUri': ('CodeGen', 69),
    'OutputUriAlsoQueryInput': ('CodeGen', 70),
    'Internal': ('CodeGen', 71),
    'DSCStreamError': ('StoreClient', 0),
    'StreamDoesNotExist': ('StoreClient', 1),
    'StreamAlreadyExists': ('StoreClient', 2),
    'AttemptToReadFromAWriteStream': ('StoreClient', 3),
    'FailedToCreateStream': ('StoreClient', 4),
    'JobToCreateTableWasCanceled': ('StoreClient', 5),
    'FailedToGetReadPathsForStream': ('StoreClient', 6),
    'CannotAccesFilePath': ('StoreClient', 7),
    'PositionNotSupported': ('StoreClient', 8),
    'GetFileSizeError': ('StoreClient', 9),
    'ReadFileError': ('StoreClient', 10),
    'UnknownCompressionScheme': ('StoreClient', 11),
    'WriteFileError': ('StoreClient', 12),
    'MultiBlockEmptyPartitionList': ('StoreClient', 13),
    'GetURINotSupported': ('StoreClient', 14),
    'SetCalcFPNotSupported': ('StoreClient', 15),
    'GetFPNotSupported': ('StoreClient', 16),
    'FailedToAllocateNewNativeBuffer': ('StoreClient', 17),
    'FailedToReadFromInputChannel': ('StoreClient', 18),
    'FailedToWriteToOutputChannel': ('StoreClient', 19),
    'MultiBlockCannotAccesFilePath': ('StoreClient', 25),
    'DryadHomeMustBeSpecified': ('JobSubmission', 0),
    'ClusterNameMustBeSpecified': ('JobSubmission', 1),
    'UnexpectedJobStatus': ('JobSubmission', 2),
    'JobStatusQueryError': ('JobSubmission', 3),
    'JobOptionNotImplemented': ('JobSubmission', 4),
    'DryadLinqJobMinMustBe2OrMore': ('JobSubmission', 5),
    'SubmissionFailure': ('JobSubmission', 6),
    'UnsupportedSchedulerType': ('JobSubmission', 7),
    'UnsupportedExecutionKind': ('JobSubmission', 8),
    'DidNotCompleteSuccessfully': ('JobSubmission', 9),
    'Binaries32BitNotSupported': ('JobSubmission', 10),
    'DistinctAttributeComparerNotDefined': ('QueryAPI', 0),
    'SerializerTypeMustBeNonNull': ('QueryAPI', 1),
    'SerializerTypeMustSupportIDryadLinqSerializer': ('QueryAPI', 2),
    'UnrecognizedOperatorName': ('QueryAPI', 3),
    'UnsupportedExpressionsType': ('QueryAPI', 7),
    'UnsupportedExpressionType': ('QueryAPI', 8),
    'IndexTooSmall': ('QueryAPI', 10),
    'MultiQueryableKeyOutOfRange': ('QueryAPI', 11),
    'IndexOutOfRange': ('QueryAPI', 12),
    'ExpressionTypeNotHandled': ('QueryAPI', 15),
    'FailedToGetStreamProps': ('QueryAPI', 16),
    'MetadataRecordType': ('QueryAPI', 17),
    'JobToCreateTableFailed': ('QueryAPI', 20),
    'OnlyAvailableForPhysicalData': ('QueryAPI', 22),
    'FileSetMustBeSealed': ('QueryAPI', 23),
    'FileSetCouldNotBeOpened': ('QueryAPI', 24),
    'FileSetMustHaveAtLeastOneFile': ('QueryAPI', 25),
    'CouldNotGetClientVersion': ('QueryAPI', 27),
    'CouldNotGetServerVersion': ('QueryAPI', 28),
    'ContextDisposed': ('QueryAPI', 29),
    'UnhandledQuery': ('QueryAPI', 30),
    'ExpressionMustBeMethodCall': ('QueryAPI', 31),
    'UntypedProviderMethodsNotSupported': ('QueryAPI', 32),
    'ErrorReadingMetadata': ('QueryAPI', 33),
    'MustStartFromContext': ('QueryAPI', 34),
    'FailedToReadFrom': ('Serialization', 0),
    'EndOfStreamEncountered': ('Serialization', 1),
    'SettingPositionNotSupported': ('Serialization', 2),
    'FingerprintDisabled': ('Serialization', 3),
    'RecordSizeMax2GB': ('Serialization', 4),
    'ReadByteNotAllowed': ('Serialization', 6),
    'ReadNotAllowed': ('Serialization', 7),
    'SeekNotSupported': ('Serialization', 8),
    'SetLengthNotSupported': ('Serialization', 9),
    'FailedToDeserialize': ('Serialization', 10),
    'ChannelCannotBeReadMoreThanOnce': ('Serialization', 11),
    'WriteNotSupported': ('Serialization', 13),
    'WriteByteNotSupported': ('Serialization', 14),
    'CannotSerializeDryadLinqQuery': ('Serialization', 15),
    'CannotSerializeObject': ('Serialization', 16),
    'GeneralSerializeFailure': ('Serialization', 17),
    'SourceOfMergesortMustBeMultiEnumerable': ('VertexRuntime', 1),
    'ThenByNotSupported': ('VertexRuntime', 2),
    'AggregateNoElements': ('VertexRuntime', 3),
    'FirstNoElementsFirst': ('VertexRuntime', 4),
    'SingleMoreThanOneElement': ('VertexRuntime', 5),
    'SingleNoElements': ('VertexRuntime', 6),
    'LastNoElements': ('VertexRuntime', 7),
    'MinNoElements': ('VertexRuntime', 8),
    'MaxNoElements': ('VertexRuntime', 9),
    'AverageNoElements': ('VertexRuntime', 10),
    'RangePartitionKeysMissing': ('VertexRuntime', 11),
    'PartitionFuncReturnValueExceedsNumPorts': ('VertexRuntime', 12),
    'FailureInExcept': ('VertexRuntime', 13),
    'FailureInIntersect': ('VertexRuntime', 14),
    'FailureInSort': ('VertexRuntime', 15),
    'RangePartitionInputOutputMismatch': ('VertexRuntime', 16),
    'KeyNotFound': ('VertexRuntime', 18),
    'TooManyItems': ('VertexRuntime', 19),
    'FailureInHashGroupBy': ('VertexRuntime', 20),
    'FailureInSortGroupBy': ('VertexRuntime', 21),
    'FailureInHashJoin': ('VertexRuntime', 22),
    'FailureInHashGroupJoin': ('VertexRuntime', 23),
    'FailureInDistinct': ('VertexRuntime', 24),
    'FailureInOperator': ('VertexRuntime', 25),
    'FailureInUserApplyFunction': ('VertexRuntime', 26),
    'FailureInOrderedGroupBy': ('VertexRuntime', 27),
    'TooManyElementsBeforeReduction': ('VertexRuntime', 33),
    'CreatingDscDataFromLocalDebugFailed': ('LocalDebug', 0),
    'UnknownError': ('Unknown', 0),
}
# The reference's message-only ``DryadLinqException(string)`` constructor leaves the code at 0
# (DryadLinqException.cs:42); raise sites that mirror such a throw use ErrorCode.Unspecified.
_UNSPECIFIED = 0


class _Codes:
    """Namespace of integer error codes: ``ErrorCode.OperatorNotSupported`` etc."""

    def __init__(self):
        for name, (cat, off) in _TABLE.items():
            setattr(self, name, CATEGORY_BASE[cat] + off)
        self.Unspecified = _UNSPECIFIED

    def name_of(self, code: int) -> str:
        for name, (cat, off) in _TABLE.items():
            if CATEGORY_BASE[cat] + off == code:
                return name
        return "Unknown"

    def category_of(self, code: int) -> str:
        base = code & 0x0F000000
        for cat, b in CATEGORY_BASE.items():
            if b == base:
                return cat
        return "Unknown"

    def all(self) -> dict:
        return {name: CATEGORY_BASE[cat] + off for name, (cat, off) in _TABLE.items()}


ErrorCode = _Codes()


class DryadLinqException(Exception):
    """Base exception: carries the DryadLINQ error code (``error_code`` / ``ErrorCode``)."""

    def __init__(self, error_code: int | str = 0, message: str = "", inner: BaseException | None = None):
        if isinstance(error_code, str):
            error_code = getattr(ErrorCode, error_code)
        self.error_code = int(error_code)
        self.inner = inner
        name = ErrorCode.name_of(self.error_code)
        super().__init__(f"[{name} 0x{self.error_code:08X}] {message}" if self.error_code else message)

    @property
    def ErrorCode(self) -> int:
        return self.error_code

    @property
    def category(self) -> str:
        return ErrorCode.category_of(self.error_code)


class DryadLinqQueryException(DryadLinqException):
    pass


class DryadLinqCodeGenException(DryadLinqException):
    pass


class DryadLinqJobException(DryadLinqException):
    """Job failure (``DryadLinqJobInfo.Wait`` raises this when the job failed or was cancelled)."""


class DryadLinqSerializationException(DryadLinqException):
    pass


class DryadLinqStoreException(DryadLinqException):
    pass


class DryadLinqVertexException(DryadLinqException):
    """A vertex program raised; carries the vertex id/version for diagnosis."""

    def __init__(self, error_code=0, message="", inner=None, vertex: str | None = None, version: int = 0):
        super().__init__(error_code, message, inner)
        self.vertex = vertex
        self.version = version


class GangAgreementError(DryadLinqVertexException):
    """A collective (gang) stage stopped before its payload exchange because some rank could not
    go on: every rank raises it alike after one small all-gather of the ranks' status, so no rank
    is left blocked inside a collective its peers never enter.  ``retryable`` is False when the
    cause is deterministic (a key range past a rank's receive capacity): a re-execution would fail
    the same way, so the gang aborts at once instead of spending MaxVertexFailures attempts."""

    def __init__(self, message: str, retryable: bool = True, ranks=()):
        super().__init__(ErrorCode.FailureInSort, message)
        self.retryable = retryable
        self.ranks = tuple(ranks)


def raise_not_supported(op: str):
    raise DryadLinqCodeGenException(ErrorCode.OperatorNotSupported, f"operator {op} is not supported")
