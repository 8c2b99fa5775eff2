{{/*
Object names: <release>-<nameOverride, default "nfd">, as NFD's own chart
builds its fullname - so a values file written for the reference's bundled
NFD chart (nfd.nameOverride, nfd.master.serviceAccount.name) names the same
objects here.
*/}}
{{- define "nfd.fullname" -}}
{{- printf "%s-%s" .Release.Name (default "nfd" .Values.nameOverride) | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "nfd.masterServiceAccount" -}}
{{- default (printf "%s-master" (include "nfd.fullname" .)) .Values.master.serviceAccount.name -}}
{{- end -}}
