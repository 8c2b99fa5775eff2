{{/* Chart name. */}}
{{- define "gfd-amd.name" -}}
{{- default .Chart.Name .Values.nameOverride | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{/* Fully qualified app name (truncated to 63 chars for DNS names). */}}
{{- define "gfd-amd.fullname" -}}
{{- if .Values.fullnameOverride -}}
{{- .Values.fullnameOverride | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- $name := default .Chart.Name .Values.nameOverride -}}
{{- if contains $name .Release.Name -}}
{{- .Release.Name | trunc 63 | trimSuffix "-" -}}
{{- else -}}
{{- printf "%s-%s" .Release.Name $name | trunc 63 | trimSuffix "-" -}}
{{- end -}}
{{- end -}}
{{- end -}}

{{- define "gfd-amd.chart" -}}
{{- printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "gfd-amd.templateLabels" -}}
app.kubernetes.io/name: {{ include "gfd-amd.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- if .Values.selectorLabelsOverride }}
{{ toYaml .Values.selectorLabelsOverride }}
{{- end }}
{{- end -}}

{{- define "gfd-amd.selectorLabels" -}}
{{- if .Values.selectorLabelsOverride -}}
{{ toYaml .Values.selectorLabelsOverride }}
{{- else -}}
{{ include "gfd-amd.templateLabels" . }}
{{- end -}}
{{- end -}}

{{- define "gfd-amd.labels" -}}
helm.sh/chart: {{ include "gfd-amd.chart" . }}
{{ include "gfd-amd.templateLabels" . }}
{{- if .Chart.AppVersion }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
{{- end }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
{{- end -}}

{{/* image:tag, tag defaulting to v<appVersion>. */}}
{{- define "gfd-amd.fullimage" -}}
{{- $tag := printf "v%s" .Chart.AppVersion -}}
{{- .Values.image.repository -}}:{{- .Values.image.tag | default $tag -}}
{{- end -}}
