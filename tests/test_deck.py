"""Input deck (.dat) parser: syntax and coercion rules of the reference
InputData class (libDEEPS2D/.. obj_data.cpp)."""
import math

import pytest

DECK = """; leading comment lines
# another
<start/Case>
<data/Nx=200>          # trailing comment
<data/Lx=0.25>
<data/Odd=-0.1735.3e7>
<data/Name=Wedge15>
<data/Bad=12abc>
;<data/Commented=1>
<table=Cp/3>
100 1000.0
200 1100.0
400 1300.0
<endtable>
<end/Case>
trailing garbage after end
"""


def test_parse_basic(native):
    d = native.InputDeck.from_string(DECK)
    assert d.name() == "Case"
    assert d.get_int("Nx") == 200
    assert d.get_float("Lx") == pytest.approx(0.25)
    assert d.get_string("Name") == "Wedge15"
    assert d.table_names() == ["Cp"]


def test_malformed_number_is_truncated_like_atof(native):
    # atof stops at the second '.', as in the reference (TestCases/Wedge.dat:208)
    d = native.InputDeck.from_string(DECK)
    assert d.get_float("Odd") == pytest.approx(-0.1735)


def test_type_checks(native):
    d = native.InputDeck.from_string(DECK)
    with pytest.raises(native.DeckError):
        d.get_int("Bad")
    with pytest.raises(native.DeckError):
        d.get_float("Name")
    with pytest.raises(native.DeckError):
        d.get_int("Missing")


def test_leading_semicolon_directive_is_not_a_comment(native):
    # strtok(buf, "#;") skips leading delimiters: ';<data/..>' is still parsed
    d = native.InputDeck.from_string(DECK)
    assert d.has("Commented")
    assert d.get_int("Commented") == 1


def test_numeric_read_rewrites_stored_value(native):
    # GetFloatVal re-formats the stored string with %g (6 significant digits)
    d = native.InputDeck.from_string(DECK.replace("0.25", "0.123456789"))
    assert d.get_float("Lx") == pytest.approx(0.123456789)
    assert d.get_string("Lx") == "0.123457"


def test_table_interpolation_and_extrapolation(native):
    d = native.InputDeck.from_string(DECK)
    x, y = d.get_table("Cp")
    assert list(x) == [100, 200, 400]
    assert d.table_eval("Cp", 150) == pytest.approx(1050.0)
    assert d.table_eval("Cp", 300) == pytest.approx(1200.0)
    # linear extrapolation with the end segments
    assert d.table_eval("Cp", 50) == pytest.approx(950.0)
    assert d.table_eval("Cp", 500) == pytest.approx(1400.0)
    assert d.table_eval("Cp", 400) == pytest.approx(1300.0)


def test_missing_start_or_end(native):
    with pytest.raises(native.DeckError):
        native.InputDeck.from_string("<data/a=1>\n")
    with pytest.raises(native.DeckError):
        native.InputDeck.from_string("<start/x>\n<data/a=1>\n")


def test_duplicate_start(native):
    with pytest.raises(native.DeckError):
        native.InputDeck.from_string("<start/x>\n<start/y>\n<end/x>\n")


def test_roundtrip_to_text(native):
    d = native.InputDeck.from_string(DECK)
    d.set("Nx", "321")
    e = native.InputDeck.from_string(d.to_text())
    assert e.get_int("Nx") == 321
    assert e.table_eval("Cp", 300) == pytest.approx(1200.0)


def test_reference_decks_parse(native):
    from tests.conftest import read_deck

    for name in ["Wedge.dat", "ObliqueShock.dat", "Step.dat", "TriplePoint.dat"]:
        d = native.InputDeck.from_string(read_deck(name))
        assert d.get_int("MaxX") > 0 and d.get_int("MaxY") > 0
        assert math.isfinite(d.get_float("CFL"))
