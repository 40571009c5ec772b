"""Coding theory layer (L5): cyclic MDS codes, FRC/AGC placement, stop rules, decode."""
from .cyclic import DecodeCache, decode_error, decode_vector, make_cyclic_B, pattern_index
from .schemes import (RULE_ALL, RULE_COUNT, RULE_FRC, RULE_PARTIAL_COUNT, RULE_PARTIAL_FRC, SCHEMES, Approx,
                      Arrival, AvoidStragg, Cyclic, FRC, Message, Naive, PartialCoded, PartialReplication,
                      Replication, Scheme, SchemeError, make_scheme, scheme_key)
