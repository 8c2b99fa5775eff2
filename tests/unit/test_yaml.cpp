// YAML/JSON reader tests (the subset config files use).
#include "config/yaml.h"
#include "test.h"

using gfd::yaml::Node;
using gfd::yaml::parse;
using gfd::yaml::to_json;

TEST(Yaml_BlockMappingScalars) {
  Node n = parse("a: 1\nb: true\nc: hello world\nd: '1'\ne: \"x\\ty\"\nf: ~\ng: 1.5\nh: 0x1f\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":1,\"b\":true,\"c\":\"hello world\",\"d\":\"1\",\"e\":\"x\\ty\",\"f\":null,\"g\":1.5,\"h\":31}"));
}

TEST(Yaml_Yaml11Booleans) {
  Node n = parse("a: yes\nb: Off\nc: on\nd: N\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":true,\"b\":false,\"c\":true,\"d\":false}"));
}

TEST(Yaml_GoYamlV2Resolution) {
  // Where go-yaml v2 (the reference's reader) and PyYAML disagree the native
  // reader follows go-yaml: y/n are booleans, an exponent needs no dot, and
  // an underflowing float is a (subnormal) number, not a string.
  Node n = parse("a: y\nb: n\nc: 1e3\nd: 1.1125369292536007e-308\ne: 1e999x\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":true,\"b\":false,\"c\":1000,\"d\":1.1125369292536007e-308,\"e\":\"1e999x\"}"));
}

TEST(Yaml_NestedAndComments) {
  Node n = parse("# header\nversion: v1 # trailing\nflags:\n  migStrategy: single\n  gfd:\n    oneshot: true\n\n    sleepInterval: 30s\n");
  EXPECT_EQ(to_json(n), std::string("{\"version\":\"v1\",\"flags\":{\"migStrategy\":\"single\",\"gfd\":{\"oneshot\":true,\"sleepInterval\":\"30s\"}}}"));
}

TEST(Yaml_SequencesAllForms) {
  Node n = parse(
      "a:\n- 1\n- two\nb:\n  - x: 1\n    y: 2\n  - x: 3\nc: [1, \"a b\", c]\nd: {k: v, n: [1,2]}\ne:\n  - - 1\n    - 2\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":[1,\"two\"],\"b\":[{\"x\":1,\"y\":2},{\"x\":3}],\"c\":[1,\"a b\",\"c\"],"
                                    "\"d\":{\"k\":\"v\",\"n\":[1,2]},\"e\":[[1,2]]}"));
}

TEST(Yaml_JsonDocument) {
  Node n = parse("{\n  \"version\": \"v1\",\n  \"flags\": {\"migStrategy\": \"none\", \"x\": [1, 2.5, false, null]}\n}\n");
  EXPECT_EQ(to_json(n), std::string("{\"version\":\"v1\",\"flags\":{\"migStrategy\":\"none\",\"x\":[1,2.5,false,null]}}"));
}

TEST(Yaml_BlockScalars) {
  Node n = parse("lit: |\n  line1\n  line2\nfold: >\n  a\n  b\nstrip: |-\n  x\n");
  EXPECT_EQ(n.get("lit")->text(), std::string("line1\nline2\n"));
  EXPECT_EQ(n.get("fold")->text(), std::string("a b\n"));
  EXPECT_EQ(n.get("strip")->text(), std::string("x"));
}

TEST(Yaml_QuotedKeysAndColonsInValues) {
  Node n = parse("\"a:b\": c\nurl: http://x:80/y\n'q''s': 'it''s'\n");
  EXPECT_EQ(n.get("a:b")->text(), std::string("c"));
  EXPECT_EQ(n.get("url")->text(), std::string("http://x:80/y"));
  EXPECT_EQ(n.get("q's")->text(), std::string("it's"));
}

TEST(Yaml_DocumentMarker) {
  Node n = parse("---\na: 1\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":1}"));
  EXPECT_TRUE(parse("").is_null());
  EXPECT_TRUE(parse("# only a comment\n").is_null());
}

TEST(Yaml_DuplicateKeysLastWins) {
  Node n = parse("a: 1\na: 2\n");
  EXPECT_EQ(n.get("a")->as_int(), static_cast<int64_t>(2));
}

TEST(Yaml_AnchorsAliasesMergeKeys) {
  Node n = parse("defaults: &d\n  replicas: 2\n  rename: x\nres:\n- <<: *d\n  name: gpu\n- *d\n");
  EXPECT_EQ(to_json(n), std::string("{\"defaults\":{\"replicas\":2,\"rename\":\"x\"},\"res\":[{\"name\":\"gpu\","
                                    "\"replicas\":2,\"rename\":\"x\"},{\"replicas\":2,\"rename\":\"x\"}]}"));
  // A quoted "<<" is an ordinary key.
  EXPECT_EQ(to_json(parse("\"<<\": 1\n")), std::string("{\"<<\":1}"));
}

TEST(Yaml_Errors) {
  EXPECT_THROW_MSG(parse("a: 1\n  b: 2\n"), "line 2");
  EXPECT_THROW_MSG(parse("a: [1, 2\n"), "flow");
  EXPECT_THROW_MSG(parse("a: *missing\n"), "unknown anchor 'missing'");
  EXPECT_THROW_MSG(parse("a: !!binary aGk=\n"), "unsupported tag !!binary");
  EXPECT_THROW_MSG(parse("a: !!int x\n"), "cannot decode string as !!int");
  EXPECT_THROW_MSG(parse("a:\n  <<: 1\n"), "map merge requires map");
  EXPECT_THROW_MSG(parse("&k a: 1\n"), "mapping keys are not supported");
  EXPECT_THROW_MSG(parse("a: 1\n---\nb: 2\n"), "multiple YAML documents");
  EXPECT_THROW_MSG(parse("a: \"unterminated\n"), "quoted scalar");
  EXPECT_THROW_MSG(parse("\ta: 1\n"), "tab");
}

TEST(Yaml_JsonPrettyPrint) {
  Node n = parse("a: 1\nb: [x]\nc: {}\n");
  EXPECT_EQ(to_json(n, 2), std::string("{\n  \"a\": 1,\n  \"b\": [\n    \"x\"\n  ],\n  \"c\": {}\n}"));
}

TEST(Yaml_UnicodeEscapes) {
  Node n = parse("a: \"\\u00b5s \\U0001F600\"\n");
  EXPECT_EQ(n.get("a")->text(), std::string("\xC2\xB5s \xF0\x9F\x98\x80"));
}
