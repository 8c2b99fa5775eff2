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

TEST(Yaml_MappingIndicatorInsidePlainValueIsAnError) {
  // ": " (or ":" at the end) ends a block plain scalar; go-yaml and PyYAML
  // reject what follows.  A ':' inside a word, or inside quotes, is text.
  for (const char* doc : {"a: b: c\n", "a: b:\n", "a: x:\ty\n", "- x: y: z\n", "a: !!str b: c\n", "a: &x b: c\n",
                          "a:\n  - b: c: d\n", "run: x | grep -q 'commit: '\n"})
    EXPECT_THROW_MSG(parse(doc), "mapping values are not allowed in this context");
  EXPECT_EQ(parse("a: http://h:80/p\n").get("a")->text(), std::string("http://h:80/p"));
  EXPECT_EQ(parse("a: b :c\n").get("a")->text(), std::string("b :c"));
  EXPECT_EQ(parse("a: 'q: r'\n").get("a")->text(), std::string("q: r"));
  EXPECT_EQ(parse("a: b #c: d\n").get("a")->text(), std::string("b"));
}

TEST(Yaml_WhatCannotStartABlockValue) {
  EXPECT_THROW_MSG(parse("a: ]\n"), "did not find expected node content");
  EXPECT_THROW_MSG(parse("a: , x\n"), "did not find expected node content");
  EXPECT_THROW_MSG(parse("a: @x\n"), "cannot start any token");
  EXPECT_THROW_MSG(parse("a: `x`\n"), "cannot start any token");
  EXPECT_THROW_MSG(parse("a: %x\n"), "cannot start any token");
  EXPECT_THROW_MSG(parse("a: - x\n"), "block sequence entries are not allowed");
  EXPECT_THROW_MSG(parse("a: ? x\n"), "mapping keys are not allowed");
  EXPECT_THROW_MSG(parse("a: | x\n"), "did not find expected comment or line break");
  // Still fine: indicators inside a word, compact nested sequences, a block
  // scalar header with a comment, "- " continuing a plain scalar.
  EXPECT_EQ(parse("a: -x\n").get("a")->text(), std::string("-x"));
  EXPECT_EQ(parse("- - a\n  - b\n").items()[0].items().size(), static_cast<size_t>(2));
  EXPECT_EQ(parse("a: | # note\n  t\n").get("a")->text(), std::string("t\n"));
  EXPECT_EQ(parse("a: b\n  - c\n").get("a")->text(), std::string("b - c"));
}

TEST(Yaml_PlainScalarFoldingAndEnds) {
  // Pinned against PyYAML (tools/yaml_diff.py found the differences).
  EXPECT_EQ(parse("a: x\n  y\n\n\n  z\n").get("a")->text(), std::string("x y\n\nz"));  // n empty lines: n newlines
  EXPECT_THROW_MSG(parse("a: x # c\n  y\n"), "could not find expected ':'");     // a comment ends the scalar
  EXPECT_THROW_MSG(parse("a: x\n  : y\n"), "mapping values are not allowed");  // ':' on a continuation line
  EXPECT_EQ(parse("a: \"d\"#c\n").get("a")->text(), std::string("d"));           // comment right after a quote
  EXPECT_EQ(parse("a: 'it''s'#c\n").get("a")->text(), std::string("it's"));
  EXPECT_EQ(parse("a: \"x#y\"\n").get("a")->text(), std::string("x#y"));
  EXPECT_THROW_MSG(parse("a: !!str ]\n"), "did not find expected node content");  // after a tag, too
  EXPECT_THROW_MSG(parse("a: |--\n  x\n"), "invalid block scalar header");       // one chomping indicator
  EXPECT_THROW_MSG(parse("a:\n  }: 1\n"), "cannot start a mapping key");
}

TEST(Yaml_DocumentMarkersOnlyAtColumnZero) {
  EXPECT_EQ(parse("a:\n  ...\n").get("a")->text(), std::string("..."));
  EXPECT_EQ(parse("a:\n  ---\n").get("a")->text(), std::string("---"));
  EXPECT_EQ(parse("a: 1\n...\n").get("a")->text(), std::string("1"));
  EXPECT_THROW_MSG(parse("a: 1\n...\nb: 2\n"), "multiple YAML documents");
}

TEST(Yaml_JsonPrettyPrint) {
  Node n = parse("a: 1\nb: [x]\nc: {}\n");
  EXPECT_EQ(to_json(n, 2), std::string("{\n  \"a\": 1,\n  \"b\": [\n    \"x\"\n  ],\n  \"c\": {}\n}"));
}

TEST(Yaml_UnicodeEscapes) {
  Node n = parse("a: \"\\u00b5s \\U0001F600\"\n");
  EXPECT_EQ(n.get("a")->text(), std::string("\xC2\xB5s \xF0\x9F\x98\x80"));
}

TEST(Yaml_DoubleQuotedEscapesAndFolding) {
  // Every escape YAML 1.1 defines (values pinned against PyYAML).
  Node n = parse("a: \"\\0\\a\\b\\t\\n\\v\\f\\r\\e\\ \\\"\\/\\\\\\N\\_\\x41\"\n");
  EXPECT_EQ(n.get("a")->text(), std::string("\0\a\b\t\n\v\f\r\x1b \"/\\\xC2\x85\xC2\xA0" "A", 18));
  // A UTF-16 surrogate pair is one code point.
  EXPECT_EQ(parse("a: \"\\ud83d\\ude00\"\n").get("a")->text(), std::string("\xF0\x9F\x98\x80"));
  // An escaped line break joins the lines; an unescaped one folds to a space,
  // an empty line to a newline - in double, single and plain scalars alike.
  EXPECT_EQ(parse("a: \"x\\\n   y\"\n").get("a")->text(), std::string("xy"));
  EXPECT_EQ(parse("a: \"one\n  two\n\n  three\"\n").get("a")->text(), std::string("one two\nthree"));
  EXPECT_EQ(parse("a: 'one\n  two'\n").get("a")->text(), std::string("one two"));
  EXPECT_EQ(parse("a: plain\n  continued\n  more\n").get("a")->text(), std::string("plain continued more"));
  EXPECT_THROW_MSG(parse("a: \"\\q\"\n"), "unknown escape character 'q'");
}

TEST(Yaml_Tags) {
  Node n = parse("a: !!str 1\nb: !!str true\nc: !!str ~\nd: !!float 2\ne: !!null ''\nf: !!str 1.5\ng: !!int '7'\n"
                 "h: !!bool 'yes'\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":\"1\",\"b\":\"true\",\"c\":\"~\",\"d\":2,\"e\":null,\"f\":\"1.5\",\"g\":7,"
                                    "\"h\":true}"));
  EXPECT_TRUE(n.get("d")->kind() == Node::Kind::Float);
  EXPECT_THROW_MSG(parse("a: !!str {k: v}\n"), "!!str");
}

TEST(Yaml_FlowCollectionsWithAnchorsTagsAndMerges) {
  Node n = parse("a: [&x 1, *x, !!str 2, !!float 3, a: 1]\nb: {<<: {m: 1}, k: *x}\nc: {<<: [{p: 1}, {q: 2}]}\n");
  EXPECT_EQ(to_json(n), std::string("{\"a\":[1,1,\"2\",3,{\"a\":1}],\"b\":{\"k\":1,\"m\":1},\"c\":{\"p\":1,\"q\":2}}"));
  EXPECT_THROW_MSG(parse("a: [1 2] x\n"), "flow");
  EXPECT_THROW_MSG(parse("a: {k: v\n"), "flow");
}

TEST(Yaml_FlowSingleQuoteEscapeKeepsScalarOpen) {
  // '' inside a single-quoted flow scalar is an escaped quote, so a bracket
  // after it is text, not the collection's end (PyYAML dumps '[ as '''[').
  EXPECT_EQ(to_json(parse("['''[']\n")), std::string("[\"'[\"]"));
  EXPECT_EQ(to_json(parse("{a: '''['}\n")), std::string("{\"a\":\"'[\"}"));
  EXPECT_EQ(to_json(parse("a: ['x''}', 'y']\n")), std::string("{\"a\":[\"x'}\",\"y\"]}"));
  EXPECT_EQ(to_json(parse("a: ['it''s',\n  'b']\n")), std::string("{\"a\":[\"it's\",\"b\"]}"));
}

TEST(Yaml_BlockScalarIndicators) {
  Node n = parse("keep: |+\n  x\n\nnext: >-\n  a\n\n  b\nind: |2\n    deep\n");
  EXPECT_EQ(n.get("keep")->text(), std::string("x\n\n"));
  EXPECT_EQ(n.get("next")->text(), std::string("a\nb"));
  EXPECT_EQ(n.get("ind")->text(), std::string("  deep\n"));
  EXPECT_THROW_MSG(parse("a: |x\n  y\n"), "invalid block scalar header");
}

TEST(Yaml_ByteOrderMarkEndMarkerEmptyCollections) {
  EXPECT_EQ(to_json(parse("\xEF\xBB\xBF" "a: 1\n")), std::string("{\"a\":1}"));
  EXPECT_EQ(to_json(parse("a: 1\n...\n")), std::string("{\"a\":1}"));
  EXPECT_EQ(to_json(parse("a: []\nb: {}\n")), std::string("{\"a\":[],\"b\":{}}"));
  EXPECT_EQ(to_json(parse("- a\n- - b\n  - c\n-\n  d: 1\n")), std::string("[\"a\",[\"b\",\"c\"],{\"d\":1}]"));
}

TEST(Yaml_IntegerPrefixesAndJsonEscapes) {
  // go-yaml v2 resolves plain integers with Go's strconv.ParseInt(s, 0, 64):
  // 0o17 is octal there (PyYAML keeps it a string; tests/test_yaml_oracle.py).
  EXPECT_EQ(to_json(parse("a: 0o17\nb: 0b101\nc: 017\n")), std::string("{\"a\":15,\"b\":5,\"c\":15}"));
  EXPECT_EQ(to_json(parse("a: \"q\\\"b\\\\c\\nd\\re\"\n")), std::string("{\"a\":\"q\\\"b\\\\c\\nd\\re\"}"));
}
