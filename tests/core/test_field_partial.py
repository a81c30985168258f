"""Parity tests for ``Field``, ``ComponentField`` and ``PartialComponent``
(reference: zookeeper/core/field_test.py, zookeeper/core/partial_component_test.py)."""

from typing import List, Optional

import pytest

from zookeeper_amd import ComponentField, Field, PartialComponent, component, configure


# --------------------------------------------------------------------------- #
# Field
# --------------------------------------------------------------------------- #


@pytest.mark.parametrize("bad_default", [[1, 2, 3], {"a": 1}, lambda x, y, z: x, lambda *a: 1])
def test_field_rejects_mutable_or_multi_arg_defaults(bad_default):
    with pytest.raises(TypeError, match="If `default` is passed to `Field`, it must be either:"):
        Field(bad_default)


def test_field_without_default():
    class Holder:
        foo: int = Field()

    assert not Holder.foo.has_default
    with pytest.raises(AttributeError, match="Field 'foo' has no default or configured value"):
        Holder.foo.get_default(Holder())


@pytest.mark.parametrize(
    "name,expected", [("i", 5), ("f", 1.2), ("b", False), ("n", None), ("t", (1, "x"))]
)
def test_immutable_defaults(name, expected):
    class Holder:
        i: int = Field(5)
        f: float = Field(1.2)
        b: bool = Field(False)
        n: Optional[int] = Field(None)
        t: tuple = Field((1, "x"))

    f = getattr(Holder, name)
    assert f.has_default
    assert f.get_default(Holder()) == expected


def test_function_defaults_with_and_without_self():
    class Holder:
        foo: int = Field(lambda: 7)
        bar: List[int] = Field(lambda self: [self.baz])
        baz = 2

    h = Holder()
    assert Holder.foo.get_default(h) == 7
    assert Holder.bar.get_default(h) == [2]


def test_field_as_decorator_takes_type_from_return_annotation():
    class Holder:
        @Field
        def pi() -> float:
            return 3.14

        @property
        def pi_value(self):
            return Holder.pi.get_default(self)

        @Field
        def power(self) -> int:
            return int(self.pi_value**self.pi_value)

    h = Holder()
    assert Holder.pi.type is float and Holder.pi.get_default(h) == 3.14
    assert Holder.power.get_default(h) == 36


def test_conflicting_annotations_are_rejected():
    with pytest.raises((TypeError, RuntimeError)):

        class Holder:
            x: int

            @Field
            def x(self) -> str:
                return "a"


def test_missing_annotation_is_rejected():
    with pytest.raises((TypeError, RuntimeError)):

        class Holder:
            x = Field(3)


def test_unregistered_field_errors():
    f = Field(5)
    assert repr(f) == "<Unregistered Field>"
    with pytest.raises(ValueError, match="This field has not been registered to a component"):
        f.has_default
    with pytest.raises(ValueError, match="This field has not been registered to a component"):
        f.get_default(object())


def test_underscore_names_are_rejected():
    # Python < 3.12 wraps errors raised in `__set_name__` in a RuntimeError.
    with pytest.raises((RuntimeError, ValueError)):

        class Holder:
            _hidden: int = Field()


def test_allow_missing_excludes_default():
    assert Field(allow_missing=True).allow_missing
    with pytest.raises(ValueError):
        Field(3.14, allow_missing=True)


def test_field_get_default_checks_host_type():
    class Holder:
        foo: int = Field(1)

    with pytest.raises(TypeError, match="`get_default` must be called with an instance"):
        Holder.foo.get_default(object())


def test_field_default_function_returning_component_is_rejected():
    @component
    class Kid:
        a: int = Field(1)

    @component
    class Holder:
        kid: object = Field(lambda: Kid())

    h = Holder()
    configure(h, {})
    with pytest.raises(TypeError, match="is returning a component instance as its default"):
        h.kid


# --------------------------------------------------------------------------- #
# ComponentField
# --------------------------------------------------------------------------- #


class Abstract:
    a: int = Field()


@component
class Concrete:
    a: int = Field(2)


def test_component_field_rejects_instances_and_other_values():
    with pytest.raises(
        TypeError,
        match="The `default` passed to `ComponentField` must be a component class, not a "
        "component instance.",
    ):
        ComponentField(Concrete())
    with pytest.raises(TypeError, match="must be either a component class or a `PartialComponent`"):
        ComponentField(int)


def test_component_field_without_default():
    class Holder:
        foo: Abstract = ComponentField()

    assert not Holder.foo.has_default
    with pytest.raises(
        AttributeError, match="ComponentField 'foo' has no default or configured component class."
    ):
        Holder.foo.get_default(Holder())


def test_component_field_class_partial_and_kwargs_defaults():
    class Holder:
        by_class: Abstract = ComponentField(Concrete)
        by_partial: Abstract = ComponentField(PartialComponent(Concrete, a=5))
        by_kwargs: Abstract = ComponentField(Concrete, a=6)

    h = Holder()
    assert isinstance(Holder.by_class.get_default(h), Concrete)
    assert Holder.by_partial.get_default(h).a == 5
    assert Holder.by_kwargs.get_default(h).a == 6
    # A fresh child every time.
    assert Holder.by_class.get_default(h) is not Holder.by_class.get_default(h)


def test_component_field_kwargs_need_default_and_allow_missing():
    with pytest.raises(TypeError, match="Keyword arguments can only be passed"):
        ComponentField(a=1, b=2)
    assert ComponentField(allow_missing=True).allow_missing
    with pytest.raises(ValueError):
        ComponentField(3.14, allow_missing=True)


def test_component_field_requires_annotation():
    with pytest.raises((TypeError, RuntimeError)):

        class Holder:
            kid = ComponentField(Concrete)


# --------------------------------------------------------------------------- #
# PartialComponent
# --------------------------------------------------------------------------- #


def make_family():
    class Kid:
        pass

    @component
    class Kid1(Kid):
        a: int = Field()
        b: str = Field("foo")

    @component
    class Kid2(Kid):
        c: float = Field(3.14)

    @component
    class Dad:
        a: int = Field(10)
        kid: Kid = ComponentField()

    return Dad, Kid1, Kid2


@pytest.mark.parametrize("not_a_component", [2.71, lambda x: x * 2, type("Plain", (), {})])
def test_partial_rejects_non_components(not_a_component):
    with pytest.raises(
        TypeError, match="The class passed to `PartialComponent` must be a component class."
    ):
        PartialComponent(not_a_component, a=3)


def test_partial_rejects_instances_and_empty_kwargs():
    _, _, Kid2 = make_family()
    with pytest.raises(
        TypeError, match="`PartialComponent` must be passed component classes, not component"
    ):
        PartialComponent(Kid2(), c=3.0)
    with pytest.raises(TypeError, match="`PartialComponent` must receive at least one keyword"):
        PartialComponent(Kid2)


def test_partial_rejects_unknown_and_mutable_kwargs():
    _, _, Kid2 = make_family()
    with pytest.raises(TypeError, match="does not correspond to any field"):
        PartialComponent(Kid2, zzz=1)
    with pytest.raises(TypeError, match="Keyword arguments passed to `PartialComponent`"):
        PartialComponent(Kid2, c=[1.0])
    p = PartialComponent(Kid2, c=1.0)
    with pytest.raises(TypeError, match="does not correspond to any field"):
        p(zzz=2)


def test_partial_with_component_class_kwarg_keeps_inheritance():
    Dad, Kid1, _ = make_family()
    d = PartialComponent(Dad, kid=Kid1)()
    configure(d, {})
    assert isinstance(d.kid, Kid1)
    assert d.kid.b == "foo" and d.kid.a == 10


def test_nested_partial_and_call_time_override():
    Dad, Kid1, _ = make_family()
    d = PartialComponent(Dad, kid=PartialComponent(Kid1, a=5))()
    configure(d, {})
    assert isinstance(d.kid, Kid1) and d.kid.a == 5
    assert PartialComponent(Kid1, a=5)(a=6).a == 6


def test_partial_lazy_function_kwarg():
    calls = []

    @component
    class Holder:
        items: list = Field(lambda: [])

    def make():
        calls.append(1)
        return [1, 2]

    p = PartialComponent(Holder, items=make)
    assert calls == []
    h = p()
    assert calls == [1] and h.items == [1, 2]


def test_partial_cannot_be_assigned_in_class_body():
    _, Kid1, _ = make_family()
    with pytest.raises((ValueError, RuntimeError)):

        class Holder:
            kid = PartialComponent(Kid1, a=1)
