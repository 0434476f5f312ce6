"""dukehip — MI355X-native Duke candidate-pair scoring behind the sesam-duke-microservice.

The product is libdukehip.so (csrc/, C-ABI in include/dukehip.h); this package is the
host-side mirror of the reference's Processor / Database / MatchListener contracts.
"""
from . import _abi
from ._abi import DukeHipError, Column
from .config import DukeConfig, Property, Comparator, parse_duke_config, parse_microservice_config
from .records import Record, KeyFunction, PartsKey, records_from_entities, parse_entities
from .processor import (GpuProcessor, GpuBlockingDatabase, GpuEngine, MatchListener,
                        CollectingListener, MatchResult)

__all__ = ["DukeHipError", "Column", "DukeConfig", "Property", "Comparator", "parse_duke_config",
           "parse_microservice_config", "Record", "KeyFunction", "PartsKey",
           "records_from_entities", "parse_entities", "GpuProcessor", "GpuBlockingDatabase",
           "GpuEngine", "MatchListener", "CollectingListener", "MatchResult", "_abi"]
